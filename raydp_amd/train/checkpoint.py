"""Directory checkpoints (``Checkpoint``) and the torch model checkpoint helper.

Format parity with the reference (``python/raydp/torch/estimator.py:254-270`` and ``:392-396``):
a checkpoint is a directory; the torch estimator writes ``model.pt`` =
``torch.save(model.state_dict())`` from rank 0, and ``TorchCheckpoint.get_model(model)`` loads
it back into the user's module. Optional ``optim.pt`` (optimizer state) supports resuming.
"""
import contextlib
import os
import pickle
import shutil
import tempfile
from typing import Any, Dict, Optional

MODEL_KEY = "model.pt"


class Checkpoint:
    def __init__(self, path: str, movable: bool = False):
        self.path = os.path.abspath(path)
        # a staging directory the framework owns (session.staging_dir): report() renames it
        # into place instead of copying it
        self._movable = movable

    @classmethod
    def from_directory(cls, path: str) -> "Checkpoint":
        return cls(path)

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "Checkpoint":
        d = tempfile.mkdtemp(prefix="raydp_ckpt_")
        with open(os.path.join(d, "dict_checkpoint.pkl"), "wb") as f:
            pickle.dump(data, f)
        return cls(d)

    def to_dict(self) -> Dict[str, Any]:
        p = os.path.join(self.path, "dict_checkpoint.pkl")
        with open(p, "rb") as f:  # written by from_dict in this framework only
            return pickle.load(f)

    def to_directory(self, path: Optional[str] = None) -> str:
        if path is None:
            return self.path
        os.makedirs(path, exist_ok=True)
        for f in os.listdir(self.path):
            src = os.path.join(self.path, f)
            if os.path.isdir(src):
                shutil.copytree(src, os.path.join(path, f), dirs_exist_ok=True)
            else:
                shutil.copy2(src, os.path.join(path, f))
        return path

    @contextlib.contextmanager
    def as_directory(self):
        yield self.path

    def get_metadata(self):
        return {}

    def __repr__(self):
        return f"Checkpoint(path={self.path})"


class TorchCheckpoint(Checkpoint):
    @classmethod
    def from_state_dict(cls, state_dict, path: Optional[str] = None):
        import torch
        d = path or tempfile.mkdtemp(prefix="raydp_torch_ckpt_")
        os.makedirs(d, exist_ok=True)
        torch.save(state_dict, os.path.join(d, MODEL_KEY))
        return cls(d)

    @classmethod
    def from_model(cls, model, path: Optional[str] = None):
        return cls.from_state_dict(model.state_dict(), path)

    def get_model(self, model=None):
        import torch
        state = torch.load(os.path.join(self.path, MODEL_KEY), map_location="cpu", weights_only=True)
        if model is None:
            raise ValueError("a model instance (or creator) is required to load a state dict")
        if callable(model) and not isinstance(model, torch.nn.Module):
            model = model({})
        if isinstance(state, torch.nn.Module):
            return state
        model.load_state_dict(state)
        return model
