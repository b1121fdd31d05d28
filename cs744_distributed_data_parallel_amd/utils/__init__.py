"""Runtime utilities: flat arenas, timers, seeding, checkpointing, tracing."""
from .arena import BufferArena, FlatArena, arena_for
from .checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint
from .seed import seed_everything
from .timer import PhaseTimer, Stopwatch

__all__ = [
    "BufferArena", "FlatArena", "arena_for", "latest_checkpoint", "load_checkpoint", "save_checkpoint",
    "seed_everything", "PhaseTimer", "Stopwatch",
]
