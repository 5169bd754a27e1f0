"""``torch.backends`` entry point (torch/__init__.py ``_import_device_backends``).

Runs at the end of ``import torch`` in every interpreter that has this package's
dist-info on ``sys.path`` -- including the fresh interpreters that
``mp.set_start_method("spawn")`` starts for the reference's workers (main.py:101-105).
It registers the ``mi355x`` backend and, when ``PDCC_TAKEOVER_GLOO=1``, makes a
literal ``init_process_group("gloo", ...)`` (main.py:90,94) use it, so main.py
runs unmodified. It never raises: a failure here would break ``import torch``.
"""


def _autoload() -> None:
    import os

    if os.environ.get("PDCC_AUTOLOAD", "1") == "0":
        return
    try:
        from .parallel.backend import register, takeover_from_env

        register()
        takeover_from_env()
    except Exception as e:  # pragma: no cover
        import sys

        print(f"[pdcc] autoload skipped: {e!r}", file=sys.stderr)
