"""Process groups (mi355x backend registration), launching, and DP helpers."""
from .backend import BACKEND_NAME, describe, install_takeover, last_algo, native_backend, register, stats  # noqa: F401
