"""Workloads: the tutorial's collective demos and a small DP model."""
from .demos import DEMOS, golden  # noqa: F401
from .mlp import MLP, synthetic_batch  # noqa: F401
