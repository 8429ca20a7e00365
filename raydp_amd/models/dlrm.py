"""DLRM (Naumov et al.; reference: the ``Dlrm`` model of examples/pytorch_dlrm.ipynb cell 9)
re-designed for MI355X: the 26 embedding tables are one fused parameter gathered by a HIP
kernel straight into the interaction input, the dot interaction runs on MFMA
(``raydp_amd.ops.dlrm_ops``), and on the GPU both MLP towers run on the fused Linear+bias+ReLU
MFMA GEMMs (``raydp_amd.ops.linear_ops``; eager ``nn.Linear`` + ``ReLU`` on the CPU).

``model_parallel=True`` shards the tables over the process group instead (table-wise, all-to-all
exchange) for multi-GPU training.

Same constructor and ``forward(*inputs)`` contract as the reference, so it drops into
``TorchEstimator`` with ``feature_columns = ['_c1', ..., '_c39']``: the first
``num_numerical_features`` inputs are float columns, the rest integer category ids.
"""
import math
from typing import Optional, Sequence

import torch
import torch.nn as nn

from raydp_amd.ops.dlrm_ops import FusedEmbeddings, dot_interaction


class TorchMlp(nn.Module):
    def __init__(self, input_dim: int, sizes: Sequence[int]):
        super().__init__()
        layers = []
        for out_dim in sizes:
            layers += [nn.Linear(input_dim, out_dim), nn.ReLU(inplace=True)]
            input_dim = out_dim
        self.layers = nn.Sequential(*layers)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, math.sqrt(2.0 / (m.in_features + m.out_features)))
                nn.init.normal_(m.bias, 0.0, math.sqrt(1.0 / m.out_features))

    @property
    def weights(self):
        return [m.weight for m in self.layers if isinstance(m, nn.Linear)]

    @property
    def linears(self):
        return [m for m in self.layers if isinstance(m, nn.Linear)]

    def forward(self, x):
        if x.is_cuda and _fused_ok(x):
            if getattr(self, "_fused", None) is None:
                from raydp_amd.ops.linear_ops import FusedLinearTower
                self._fused = FusedLinearTower(self.linears, [True] * len(self.linears), out_f32=True)
            return self._fused(x)
        return self.layers(x)


def _fused_ok(x) -> bool:
    from raydp_amd.ops.linear_ops import tower_enabled
    return x.dim() == 2 and x.dtype in (torch.float32, torch.bfloat16) and tower_enabled()


class Dlrm(nn.Module):
    def __init__(self, num_numerical_features: int, categorical_feature_sizes: Sequence[int],
                 bottom_mlp_sizes: Sequence[int], top_mlp_sizes: Sequence[int], embedding_dim: int = 32,
                 fused_embedding_sgd_lr: Optional[float] = None, model_parallel: bool = False,
                 embedding_group=None, static_batch="auto"):
        super().__init__()
        if embedding_dim != bottom_mlp_sizes[-1]:
            raise ValueError("The last bottom MLP layer must have same size as embedding.")
        self.num_numerical_features = num_numerical_features
        self.embedding_dim = embedding_dim
        self.bottom_mlp = TorchMlp(num_numerical_features, bottom_mlp_sizes)
        if model_parallel:
            # table-wise sharding over the process group, all-to-all of ids / rows
            # (raydp_amd.parallel.embedding_mp); the MLPs stay data parallel
            from raydp_amd.parallel.embedding_mp import ShardedEmbeddings
            self.embeddings = ShardedEmbeddings(categorical_feature_sizes, embedding_dim, group=embedding_group,
                                                fused_sgd_lr=fused_embedding_sgd_lr, static_batch=static_batch)
        else:
            self.embeddings = FusedEmbeddings(categorical_feature_sizes, embedding_dim, fused_embedding_sgd_lr)
        f = len(categorical_feature_sizes) + 1
        self.num_interactions = embedding_dim + f * (f - 1) // 2 + 1
        self.top_mlp = TorchMlp(self.num_interactions, top_mlp_sizes[:-1])
        self.out = nn.Linear(top_mlp_sizes[-2], top_mlp_sizes[-1])
        with torch.no_grad():   # the zero-pad column of the interaction never contributes
            self.top_mlp.weights[0][:, -1].zero_()

    def forward(self, *inputs):
        ntab = len(self.embeddings.table_sizes)
        if len(inputs) == 2 and inputs[0].dim() == 2 and inputs[0].shape[1] == self.num_numerical_features \
                and inputs[1].dim() == 2 and inputs[1].shape[1] == ntab and ntab + self.num_numerical_features != 2:
            dense, cats = inputs      # (dense [B, 13], categorical ids [B, 26])
        else:
            dense = torch.cat(inputs[:self.num_numerical_features], dim=1).float()
            cats = torch.cat(inputs[self.num_numerical_features:], dim=1)
        pending = None
        if hasattr(self.embeddings, "start"):
            # sharded tables: the id all-to-all is in flight while the bottom MLP runs
            pending = self.embeddings.start(cats)
        mlp_out = self.bottom_mlp(dense.float())
        if pending is not None:
            Z = dot_interaction(self.embeddings.finish(pending, mlp_out))
        else:   # replicated tables: lookup + interaction fused (one kernel each way on the GPU)
            Z = self.embeddings.interact(mlp_out, cats.long(), relu_head=True)   # TorchMlp ends in ReLU
        if Z.is_cuda and _fused_ok(Z):
            # the whole top tower including the output layer is one fused op: the last bf16
            # activation never leaves the chain and the logits come back fp32
            if getattr(self, "_top_fused", None) is None:
                from raydp_amd.ops.linear_ops import FusedLinearTower
                lins = self.top_mlp.linears + [self.out]
                self._top_fused = FusedLinearTower(lins, [True] * (len(lins) - 1) + [False], out_f32=True)
            return self._top_fused(Z)
        return self.out(self.top_mlp(Z))
