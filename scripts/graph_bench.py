"""Per-step time of TorchLoopEngine on the stroke tutorial's NET_Model: eager vs HIP-graph replay
(chunk sizes), synthetic data of the tutorial's shape (4611 rows x 11 feature columns, batch 64).

    python scripts/graph_bench.py [--epochs 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tutorials"))

from stroke import NET_Model  # noqa: E402

from raydp_amd.torch.engine import TorchLoopEngine  # noqa: E402
from raydp_amd.torch.metrics import TorchMetric  # noqa: E402
from raydp_amd.train import session  # noqa: E402


class _Shard:
    def __init__(self, feats, labels):
        self.feats, self.labels, self.n, self.multi = feats, labels, labels.shape[0], True


def run(mode, chunk, epochs, n=4611, batch=64):
    os.environ["RAYDP_TORCH_GRAPHS"] = "0" if mode.startswith("eager") else "1"
    os.environ["RAYDP_TORCH_GRAPH_CHUNK"] = str(chunk)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = NET_Model(11)
    if mode.endswith("fused"):
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=(mode != "eager_nocap"))
    cfg = {"batch_size": batch, "shuffle": True, "drop_last": False}
    session._set_session(session._Session(session.TrainContext(), {}, lambda *a: None, "/tmp"))
    e = TorchLoopEngine(model, opt, nn.SmoothL1Loss(), TorchMetric(["Accuracy"]), dev, cfg, None)
    g = torch.Generator().manual_seed(1)
    cards = [2, 0, 2, 2, 2, 5, 2, 0, 0, 4, 5]   # NET_Model.sparse_idx -> embedding sizes
    feats = [(torch.randint(0, max(c, 2), (n, 1), generator=g).float() if c else torch.randn(n, 1, generator=g)).to(dev)
             for c in cards]
    for emb, col in zip(model.embs, model.sparse_idx):   # host-side bounds check before any launch
        assert int(feats[col].max()) < emb.num_embeddings, (col, emb.num_embeddings)
    lab = (torch.rand(n, generator=g) > 0.5).float().to(dev)
    e.train = _Shard(feats, lab)
    ts = []
    for _ in range(epochs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.train_epoch()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    session._set_session(None)
    med = statistics.median(ts[2:])
    steps = -(-n // batch)
    return {"mode": mode, "chunk": chunk, "epoch_s": round(med, 5), "us_per_step": round(med / steps * 1e6, 1),
            "engine": e.name, "graph_failed": getattr(e.graphed, "failed", None)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--modes", default="eager_nocap:1,eager:1,graph:1,graph:8,graph:32")
    a = ap.parse_args()
    for m in a.modes.split(","):
        mode, chunk = m.split(":")
        print(json.dumps(run(mode, int(chunk), a.epochs)), flush=True)


if __name__ == "__main__":
    main()
