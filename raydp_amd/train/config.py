"""Ray-Train-compatible configuration objects (ScalingConfig / RunConfig / FailureConfig).

Reference use: ``python/raydp/torch/estimator.py:331-334``.
"""
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class ScalingConfig:
    num_workers: int = 1
    use_gpu: Optional[bool] = None          # None: use GPUs when present
    resources_per_worker: Optional[Dict[str, float]] = None
    placement_strategy: Any = "PACK"
    trainer_resources: Optional[Dict[str, float]] = None

    def gpus_per_worker(self) -> float:
        if self.resources_per_worker and "GPU" in self.resources_per_worker:
            return float(self.resources_per_worker["GPU"])
        return 1.0 if self.use_gpu else 0.0


@dataclass
class FailureConfig:
    max_failures: int = 0
    fail_fast: bool = False


@dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_frequency: int = 0
    checkpoint_at_end: Optional[bool] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"


@dataclass
class RunConfig:
    name: Optional[str] = None
    storage_path: Optional[str] = None
    failure_config: FailureConfig = field(default_factory=FailureConfig)
    checkpoint_config: CheckpointConfig = field(default_factory=CheckpointConfig)
    verbose: int = 0
