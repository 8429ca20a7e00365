"""Fusable-model recognition (raydp_amd/models/mlp_spec.py), incl. the embedding front of the
stroke tutorial's NET_Model, and the fused trainer's host-side layout of such a model (no GPU)."""
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

from raydp_amd.models.mlp_spec import extract_mlp_spec

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tutorials"))
from stroke import NET_Model  # noqa: E402


class Front(nn.Module):
    def __init__(self, emb=None, share=False):
        super().__init__()
        self.e1 = emb or nn.Embedding(4, 3)
        self.e2 = self.e1 if share else nn.Embedding(6, 2)
        self.fc1, self.fc2 = nn.Linear(2 + 3 + 2, 32), nn.Linear(32, 1)

    def forward(self, x):
        z = torch.cat([x[:, [0, 3]], self.e1(x[:, 1].long()), self.e2(x[:, 2].long())], dim=1)
        return self.fc2(F.relu(self.fc1(z)))


def test_stroke_net_model_has_an_embedding_front():
    spec = extract_mlp_spec(NET_Model(11))
    assert spec is not None and len(spec.layers) == 5
    assert spec.raw_features == 11
    assert [c.src for c in spec.front] == [1, 7, 8, 0, 2, 3, 4, 5, 6, 9, 10]
    assert [c.emb is None for c in spec.front] == [True] * 3 + [False] * 8
    assert len(spec.embeddings()) == 8


def test_front_columns_follow_embedding_dims():
    m = Front()
    spec = extract_mlp_spec(m)
    assert spec is not None
    assert [(c.src, c.emb is m.e1, c.emb is m.e2, c.j) for c in spec.front] == [
        (0, False, False, 0), (3, False, False, 0), (1, True, False, 0), (1, True, False, 1),
        (1, True, False, 2), (2, False, True, 0), (2, False, True, 1)]
    # a second instance of the same structure is rebuilt from the cached recipe
    m2 = Front()
    spec2 = extract_mlp_spec(m2)
    assert [c.emb is m2.e1 for c in spec2.front] == [c.emb is m.e1 for c in spec.front]


def test_plain_mlp_has_no_front():
    m = nn.Sequential(nn.Linear(5, 8), nn.ReLU(), nn.Linear(8, 1))
    spec = extract_mlp_spec(m)
    assert spec is not None and spec.front is None and spec.raw_features is None


def test_unsupported_fronts_fall_back():
    assert extract_mlp_spec(Front(emb=nn.Embedding(4, 3, padding_idx=0))) is None
    assert extract_mlp_spec(Front(emb=nn.Embedding(300, 3))) is None       # ids must be exact in bf16

    class Shared(Front):
        def __init__(self):
            super().__init__()
            self.e2 = nn.Embedding(4, 3)
            self.fc1 = nn.Linear(2 + 3 + 3, 32)

        def forward(self, x):   # one table looked up by two columns: gradients would collide
            z = torch.cat([x[:, [0, 3]], self.e1(x[:, 1].long()), self.e1(x[:, 2].long())], dim=1)
            return self.fc2(F.relu(self.fc1(z)))
    assert extract_mlp_spec(Shared()) is None


def test_fused_layout_of_front_model():
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    m = NET_Model(11)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    tr = FusedMLPTrainer(extract_mlp_spec(m), optimizer_config(opt), loss_code(nn.SmoothL1Loss()), 64, None,
                         layout_only=True, acc_thr=0.5)
    d = tr.desc
    assert d.front_n == 11 and d.acc_mode == 1 and tr.feat_k == 16
    assert d.front_q == 2 + 2 + 2 + 2 + 5 + 2 + 4 + 5
    emb = [(k, mod, off, n) for k, mod, off, n in tr.layout if k == "emb"]
    assert len(emb) == 8
    for k in range(3, 11):
        fc = d.front[k]
        e = m.embs[k - 3]
        off = [o for _, mod, o, _ in emb if mod is e][0]
        assert (fc.poff, fc.stride, fc.rows, fc.src) == (off, 1, e.num_embeddings, m.sparse_idx[k - 3])
        assert torch.equal(tr.params[off:off + e.num_embeddings], e.weight.detach().reshape(-1))
    assert [d.front[k].poff for k in range(3)] == [-1, -1, -1]
