"""ddq -- MI355X-native data-parallel DQN step (drop-in for defc0n1/distributed-deep-q's
worker/param-server hot path).  Compute lives in libddq_hip.so (hand-written HIP for
gfx950); this package mirrors the reference's Python operator surface."""
from ._lib import DDQError  # noqa: F401
from .net import DeepQNet, GAMMA, NUM_ACTIONS, NFRAME  # noqa: F401

__version__ = "0.1.0"
