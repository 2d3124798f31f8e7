"""gym_cooking_amd -- MI355X-native batched step engine for the Overcooked kitchen of
deletfsi/gym-cooking (environment step + planner rollout hot path).

Modules:
  levels  -- level parsing / builtin kitchens / recipe goal masks (host)
  capi    -- ctypes binding of include/oc_engine.h (liboc_engine.so)
  engine  -- OvercookedBatch: torch-buffer batched reset/step on one GPU
  envs    -- OvercookedEnvironment: the gym-surface drop-in (one env of a batch)
  dist    -- one-process-per-GPU sharding + RCCL all-gather of episode summaries
"""
from . import levels  # noqa: F401

__all__ = ["levels"]
__version__ = "0.1.0"
