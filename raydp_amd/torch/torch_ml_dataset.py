"""Legacy data adapters of the reference's torch package, re-built on this framework's Dataset
(reference: python/raydp/torch/torch_ml_dataset.py:30-111, written against the removed
``ray.util.data.MLDataset``).

* ``TorchMLDataset``: an ``IterableDataset`` that yields ``collate_fn(pandas_block)`` per block
  of a :class:`raydp_amd.data.Dataset` (optionally shuffling each block with a fixed seed);
  ``len()`` is the row count (from block metadata, no pass over the data).
* ``PrefetchedDataLoader``: a background thread pulls batches from a base loader into a
  bounded queue. With ``device=`` it also moves every tensor of a batch to the GPU with
  ``non_blocking`` copies on a side stream and hands the batch over with an event, so the
  host->HBM copy of batch k+1 overlaps compute on batch k (the "device-side prefetch queue"
  SURVEY.md §2.2 P15 calls for).
"""
import logging
import queue
import threading
from typing import Callable, Optional

import torch
from torch.utils.data import IterableDataset

logger = logging.getLogger(__name__)


class TorchMLDataset(IterableDataset):
    def __init__(self, ds, collate_fn: Callable, shuffle: bool = False, shuffle_seed: Optional[int] = None):
        super().__init__()
        self.ds = ds
        self.collate_fn = collate_fn
        self.shuffle = shuffle
        self.shuffle_seed = shuffle_seed or 1

    def __iter__(self):
        for t in self.ds._get_tables():
            pdf = t.to_pandas()
            if self.shuffle:
                pdf = pdf.sample(frac=1.0, random_state=self.shuffle_seed)
            yield self.collate_fn(pdf)

    def __len__(self):
        return self.ds.count()


def _to_device(obj, device, stream):
    if isinstance(obj, torch.Tensor):
        src = obj.pin_memory() if obj.device.type == "cpu" and device.type == "cuda" else obj
        return src.to(device, non_blocking=True)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_device(o, device, stream) for o in obj)
    if isinstance(obj, dict):
        return {k: _to_device(v, device, stream) for k, v in obj.items()}
    return obj


class PrefetchedDataLoader:
    _END = object()

    def __init__(self, base_loader, max_size: int = 5, device=None):
        self.base_loader = base_loader
        self.max_size = max_size
        self.device = torch.device(device) if device is not None else None
        self.queue = None
        self.fetcher = None
        self.fetcher_stop = threading.Event()
        self._error = None

    def _stop_fetcher(self):
        if self.fetcher is not None:
            self.fetcher_stop.set()
            while self.fetcher.is_alive():   # unblock a producer waiting on a full queue
                try:
                    self.queue.get_nowait()
                except queue.Empty:
                    pass
                self.fetcher.join(timeout=0.01)
        self.fetcher = None
        self.fetcher_stop.clear()

    def _setup(self):
        self._stop_fetcher()
        self.queue = queue.Queue(maxsize=self.max_size)
        self._error = None
        it = iter(self.base_loader)
        cuda = self.device is not None and self.device.type == "cuda"
        stream = torch.cuda.Stream(device=self.device) if cuda else None

        def fetch_task():
            try:
                while not self.fetcher_stop.is_set():
                    try:
                        item = next(it)
                    except StopIteration:
                        break
                    ev = None
                    if self.device is not None:
                        if cuda:
                            with torch.cuda.stream(stream):
                                item = _to_device(item, self.device, stream)
                                ev = torch.cuda.Event()
                                ev.record(stream)
                        else:
                            item = _to_device(item, self.device, None)
                    self.queue.put((item, ev))
            except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
                self._error = e
            finally:
                self.queue.put((self._END, None))
        self.fetcher = threading.Thread(target=fetch_task, daemon=True, name="raydp-prefetch")
        self.fetcher.start()

    def __iter__(self):
        self._setup()
        while True:
            item, ev = self.queue.get()
            if item is self._END:
                break
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
            yield item
        if self._error is not None:
            raise self._error

    def __len__(self):
        return len(self.base_loader)
