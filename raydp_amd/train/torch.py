"""``ray.train.torch`` equivalents: ``TorchTrainer``, ``prepare_model``, ``TorchCheckpoint``,
``TorchConfig``."""
from raydp_amd.train.checkpoint import TorchCheckpoint  # noqa: F401
from raydp_amd.train.trainer import TorchTrainer, prepare_model  # noqa: F401


def get_device():
    from raydp_amd.train.session import get_device as _gd
    return _gd()


def prepare_data_loader(data_loader, move_to_device=True):
    return data_loader
