"""MI355X-native two-tower training step (drop-in for DiegoPaniagua23/
music-recommendation-multimodal ``src/models`` + the ``src/train.py`` InfoNCE loop).

Import with ``importlib.import_module("music-recommendation-multimodal_amd")`` (the
directory name is not a Python identifier).  Kernels live in ``lib/libttmi.so`` (C ABI:
``include/ttmi.h``), built by ``make`` / ``__graft_entry__.build()``.
"""
from . import lib
from . import ops
from . import functional
from . import cnn
from . import text
from . import retrieval
from . import preprocess
from . import data
from .data import MultimodalDataset, DeviceCollator, DevicePrefetcher
from .text import TextEncoder
from .user_tower import SequentialUserEncoder
from .item_tower import MultimodalItemEncoder
from .two_tower import TwoTowerModel, infonce, infonce_global
from .train import (FlatParams, GradSync, TrainStep, cleanup_ddp, setup_ddp,
                    train_one_epoch)

__all__ = ["lib", "ops", "functional", "cnn", "SequentialUserEncoder", "MultimodalItemEncoder",
           "TwoTowerModel", "infonce", "infonce_global", "TrainStep", "FlatParams", "GradSync", "setup_ddp",
           "cleanup_ddp", "train_one_epoch", "preprocess", "data", "MultimodalDataset", "DeviceCollator",
           "DevicePrefetcher"]
