"""MI355X-native collective communication for PyTorch.

Same capabilities and Python API as the ``torch.distributed`` collectives
tutorial it is modelled on (reference ``main.py``: ``reduce``, ``all_reduce``,
``scatter``, ``gather``, ``all_gather``, ``broadcast`` with
``ReduceOp.SUM/PRODUCT/MAX/MIN``, ``init_process_group``/``new_group`` and a
``torch.multiprocessing`` spawn launcher), served by a native c10d backend
(``mi355x``) built for gfx950:

* GPU tensors: hipIpc peer-memory collectives with hand-written CDNA4 kernels
  (LDS-DMA staged N-way reduce, multi-tensor pack/unpack, xGMI pulls,
  cross-GPU flags) for small/medium messages; RCCL called directly for bulk;
* CPU tensors: a POSIX shared-memory host transport.

Quick start::

    import pytorch_distributed_collective_communication_amd.distributed as dist
    dist.init_process_group("gloo", rank=r, world_size=n)   # served by mi355x
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
"""
from __future__ import annotations

import importlib
import os

__version__ = "0.1.0"

_native_mod = None


def _load_native():
    """Import the in-tree native extension ``_C``; fail loudly if it is missing."""
    global _native_mod
    if _native_mod is None:
        so = os.environ.get("PDCC_NATIVE_SO")  # another build of _C (the sanitized one, tests/test_sanitizers.py)
        if so:
            import sys
            from importlib import util as _util

            spec = _util.spec_from_file_location(__name__ + "._C", so)
            if spec is None or not os.path.exists(so):
                raise ImportError(f"PDCC_NATIVE_SO={so}: no such extension")
            mod = _util.module_from_spec(spec)
            sys.modules[__name__ + "._C"] = mod
            spec.loader.exec_module(mod)
            _native_mod = mod
            return _native_mod
        try:
            _native_mod = importlib.import_module(__name__ + "._C")
        except ImportError as e:  # pragma: no cover - exercised only on broken installs
            raise ImportError(
                "pytorch_distributed_collective_communication_amd: native extension _C is not built. "
                "Run `python -m pytorch_distributed_collective_communication_amd._build` "
                f"(needs hipcc for gfx950). Original error: {e}"
            ) from e
    return _native_mod


def native_available() -> bool:
    try:
        _load_native()
        return True
    except ImportError:
        return False


from .parallel.backend import BACKEND_NAME, install_takeover, register  # noqa: E402

register()
if os.environ.get("PDCC_TAKEOVER_GLOO", "0") not in ("", "0") or os.environ.get(
    "PDCC_TAKEOVER_NCCL", "0"
) not in ("", "0"):
    from .parallel.backend import takeover_from_env

    takeover_from_env()

__all__ = ["BACKEND_NAME", "register", "install_takeover", "native_available", "__version__"]
