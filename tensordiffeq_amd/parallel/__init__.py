"""Distributed execution (reference: MirroredStrategy DP, models.py:230-277, fit.py:150-224)."""
from .dist import (DistContext, init_distributed, get_context, reset_context, shard_range, shard,
                   destroy, env_world)

__all__ = ["DistContext", "init_distributed", "get_context", "reset_context", "shard_range",
           "shard", "destroy", "env_world"]
