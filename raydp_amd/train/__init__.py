"""Worker-group training (Ray Train equivalent)."""
from raydp_amd.train.checkpoint import Checkpoint, TorchCheckpoint
from raydp_amd.train.config import CheckpointConfig, FailureConfig, RunConfig, ScalingConfig
from raydp_amd.train.session import (get_checkpoint, get_context, get_dataset_shard, get_device,
                                     get_local_rank, get_world_rank, get_world_size, report)
from raydp_amd.train.trainer import (DataParallelTrainer, Result, TorchTrainer,
                                     TrainingFailedError, prepare_model)

__all__ = ["Checkpoint", "TorchCheckpoint", "CheckpointConfig", "FailureConfig", "RunConfig",
           "ScalingConfig", "get_checkpoint", "get_context", "get_dataset_shard", "get_device",
           "get_local_rank", "get_world_rank", "get_world_size", "report", "DataParallelTrainer",
           "Result", "TorchTrainer", "TrainingFailedError", "prepare_model"]

from raydp_amd.train import torch  # noqa: E402,F401  (ray.train.torch)
