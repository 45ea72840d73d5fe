"""ggrs_amd -- MI355X batched rollback-resimulation engine for GGRS's hot path.

The engine replays GGRS's LoadGameState -> N x AdvanceFrame -> SaveGameState program (SyncLayer /
SyncTestSession, caspark/ggrs 0.10.2) for thousands of (session, branch) lanes at once, with
hand-written HIP kernels for gfx950 behind a C ABI (include/ggrs_amd.h).  See DESIGN.md.
"""
from ._lib import GgrsError, InvalidRequest, PreconditionError, NULL_FRAME  # noqa: F401
from .session import (AdvanceFrame, BoxGameHandler, Engine, LaneBatch, LaneBoxGameHandler,  # noqa: F401
                      LanesFailed, LoadGameState, MismatchedChecksum, SaveGameState, SessionBuilder,
                      SyncTestSession, encode_lane_lists)

from .handler import BatchedHandler, GameStateCell  # noqa: F401
from .branch import BranchEngine  # noqa: F401
from .particles import ParticleEngine  # noqa: F401
from .p2p import P2PEngine  # noqa: F401

__version__ = "0.1.0"
