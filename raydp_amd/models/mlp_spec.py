"""Recognise fusable MLPs in user ``nn.Module``s (torch.fx pattern match).

A model qualifies for the fused HIP trainer when its traced graph is a single chain of
``Linear`` layers, each hidden one followed by an optional activation (ReLU / identity) and an
optional ``BatchNorm1d`` in either order, ending in a bare ``Linear``. That covers the
reference's ``NYC_Model`` (``examples/pytorch_nyctaxi.py:69-92``: Linear→ReLU→BN ×4 →
Linear), the ``LinearModel`` of ``tests/test_torch.py`` and DLRM-style MLP towers.
The chain may sit behind an *embedding front*: the model's raw input columns (``torch.cat`` of
its inputs), some copied (``x[:, [1, 7, 8]]``) and some turned into ids (``x[:, i].long()``)
and looked up in per-column ``nn.Embedding`` tables, concatenated into the first Linear's
input -- the stroke tutorial's ``NET_Model`` (reference ``tutorials/pytorch_example.ipynb``
cell 32). The fused kernel gathers those embedding rows itself (``csrc/hip/mlp_core.h``
load_front / front_backward).
Anything else (dropout, residuals, custom ops, embeddings anywhere else) returns ``None`` and
the generic device-resident PyTorch loop is used instead.
"""
import operator
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LayerSpec:
    linear: nn.Linear
    act: int = 0        # 0 identity, 1 relu
    bn: int = 0         # 0 none, 1 act->bn, 2 bn->act
    bn_module: Optional[nn.BatchNorm1d] = None


@dataclass
class FrontCol:
    src: int                                  # raw input column
    emb: Optional[nn.Embedding] = None        # None: dense copy of the column
    j: int = 0                                # element of the embedding row


@dataclass
class MlpSpec:
    layers: List[LayerSpec] = field(default_factory=list)
    front: Optional[List[FrontCol]] = None    # None: the raw input feeds the first Linear

    @property
    def raw_features(self) -> Optional[int]:
        """Raw input columns the model needs (None: exactly the first Linear's inputs)."""
        if self.front is None:
            return None
        return max(c.src for c in self.front) + 1

    def embeddings(self) -> List[nn.Embedding]:
        out: List[nn.Embedding] = []
        for c in self.front or []:
            if c.emb is not None and all(c.emb is not e for e in out):
                out.append(c.emb)
        return out

    @property
    def in_features(self):
        return self.layers[0].linear.in_features

    @property
    def out_features(self):
        return self.layers[-1].linear.out_features


_RELU_FUNCS = {F.relu, torch.relu, torch.nn.functional.relu}


_SPEC_CACHE = {}   # structural key -> recipe [(linear name, act, bn, bn name)] or None


def _structure_key(model: nn.Module):
    # by class *name* + forward code object, not the class object: models are often defined
    # inside a function, which makes a new (identical) class per call
    f = type(model).forward
    fwd = getattr(f, "__code__", None)
    cells = tuple(repr(c.cell_contents) for c in (getattr(f, "__closure__", None) or ()))
    leaves = tuple((n, type(m).__qualname__, repr(m)) for n, m in model.named_modules()
                   if not any(True for _ in m.children()))
    return type(model).__module__, type(model).__qualname__, fwd, cells, leaves


def extract_mlp_spec(model: nn.Module) -> Optional[MlpSpec]:
    """The fusable-MLP spec of ``model`` or None. The fx trace runs once per model structure
    (class, forward code, leaf modules and their hyper-parameters): a new instance of a seen
    structure is rebuilt from the cached recipe (the trace costs ~2 ms per fit)."""
    try:
        key = _structure_key(model)
        hash(key)
    except Exception:  # noqa: BLE001
        key = None
    if key is not None and key in _SPEC_CACHE:
        recipe = _SPEC_CACHE[key]
        if recipe is None:
            return None
        layers, front = recipe
        spec = MlpSpec()
        for lin, act, bn, bn_name in layers:
            spec.layers.append(LayerSpec(linear=model.get_submodule(lin), act=act, bn=bn,
                                         bn_module=model.get_submodule(bn_name) if bn_name else None))
        if front is not None:
            spec.front = [FrontCol(src, model.get_submodule(e) if e else None, j) for src, e, j in front]
        return spec
    spec = _trace_spec(model)
    if key is not None:
        if len(_SPEC_CACHE) > 256:
            _SPEC_CACHE.clear()
        if spec is None:
            _SPEC_CACHE[key] = None
        else:
            names = {id(m): n for n, m in model.named_modules()}
            _SPEC_CACHE[key] = ([(names[id(ly.linear)], ly.act, ly.bn,
                                  names[id(ly.bn_module)] if ly.bn_module is not None else None)
                                 for ly in spec.layers],
                                None if spec.front is None else
                                [(c.src, names[id(c.emb)] if c.emb is not None else None, c.j) for c in spec.front])
    return spec


def _trace_spec(model: nn.Module) -> Optional[MlpSpec]:
    try:
        import torch.fx as fx
        gm = fx.symbolic_trace(model)
    except Exception:  # noqa: BLE001 - untraceable models are simply not fused
        return None
    mods = dict(gm.named_modules())
    spec = MlpSpec()
    cur = None          # current LayerSpec being extended
    prev_node = None
    placeholder = None
    sym = {}            # front world: node -> symbolic value (see _front_value)
    for node in gm.graph.nodes:
        if node.op == "placeholder":
            if placeholder is not None:
                return None  # multi-input models are not MLP chains
            placeholder = node
            prev_node = node
            sym[node] = ("in", None)
            continue
        if not spec.layers and node.op != "output" and not (
                node.op == "call_module" and isinstance(mods.get(node.target), nn.Linear)):
            # before the first Linear: column selections, id casts, embedding lookups, cats
            v = _front_value(node, sym, mods)
            if v is None:
                return None
            sym[node] = v
            prev_node = node
            continue
        if not spec.layers and node.op == "call_module":
            # the first Linear: its input is the raw input or an embedding front
            src = sym.get(node.args[0]) if node.args else None
            if src is None:
                return None
            if src != ("in", None):
                front = _front_columns(src)
                if front is None:
                    return None
                spec.front = front
            prev_node = node.args[0]
        if node.op == "output":
            if node.args[0] is not prev_node:
                return None
            break
        # every op must consume the previous op's output (a single chain)
        if not node.args or node.args[0] is not prev_node:
            return None
        if node.op == "call_module":
            m = mods[node.target]
            if isinstance(m, nn.Linear):
                cur = LayerSpec(linear=m)
                spec.layers.append(cur)
            elif isinstance(m, nn.ReLU):
                if cur is None or cur.act:
                    return None
                cur.act = 1
                if cur.bn:
                    cur.bn = 2
            elif isinstance(m, nn.BatchNorm1d):
                if cur is None or cur.bn or not m.track_running_stats or m.momentum is None:
                    return None
                cur.bn_module = m
                cur.bn = 1 if cur.act else 2
                if not cur.act:
                    cur.bn = 2  # provisional: BN first; becomes act-after if a ReLU follows
            elif isinstance(m, (nn.Identity,)):
                pass
            elif isinstance(m, nn.Dropout) and m.p == 0.0:
                pass
            else:
                return None
        elif node.op == "call_function":
            if node.target in _RELU_FUNCS and len(node.args) == 1 and not node.kwargs.get("inplace", False):
                if cur is None or cur.act:
                    return None
                cur.act = 1
            else:
                return None
        elif node.op == "call_method":
            if node.target == "relu" and len(node.args) == 1:
                if cur is None or cur.act:
                    return None
                cur.act = 1
            else:
                return None
        else:
            return None
        prev_node = node
    if not spec.layers:
        return None
    # fix BN/act order: bn==2 means BN came before the activation (or no activation)
    last = spec.layers[-1]
    if last.act or last.bn:
        return None
    for ly in spec.layers:
        if ly.bn and not ly.act:
            ly.bn = 2
    for a, b in zip(spec.layers[:-1], spec.layers[1:]):
        if a.linear.out_features != b.linear.in_features:
            return None
    for ly in spec.layers:
        if ly.linear.in_features > 512 or ly.linear.out_features > 512:
            return None
    if len(spec.layers) > 8:
        return None
    if spec.front is not None:
        if len(spec.front) != spec.layers[0].linear.in_features or len(spec.front) > 64:
            return None
        embs = spec.embeddings()
        for e in embs:
            # ids travel as bf16 features (exact below 256); torch-only options stay on torch
            if (e.num_embeddings > 256 or e.padding_idx is not None or e.max_norm is not None
                    or e.sparse or e.scale_grad_by_freq):
                return None
            # every table element must belong to exactly one front column (its gradient is stored,
            # not accumulated, by the kernel)
            cols = [(c.src, c.j) for c in spec.front if c.emb is e]
            if sorted(c[1] for c in cols) != list(range(e.embedding_dim)) or len({c[0] for c in cols}) != 1:
                return None
    return spec


def _front_value(node, sym, mods):
    """Symbolic value of a node in front of the first Linear, or None when unsupported.

    ("in", cols)      [B, k] raw input columns (cols None = all of them, in order)
    ("col", c)        [B] raw column c
    ("icol", c)       [B] raw column c cast to an integer id
    ("emb", module, c) [B, dim] embedding rows selected by raw column c
    ("front", parts)  [B, k] concatenation of "in" / "emb" parts
    """
    args = node.args
    if node.op == "call_function" and node.target is torch.cat:
        seq = args[0] if args else node.kwargs.get("tensors")
        dim = args[1] if len(args) > 1 else node.kwargs.get("dim", 0)
        if dim not in (1, -1):
            return None
        if isinstance(seq, fx_node_type()):
            # torch.cat(x) of the varargs tuple: the raw input columns
            return ("in", None) if sym.get(seq) == ("in", None) else None
        parts = []
        for a in seq:
            v = sym.get(a)
            if v is None or v[0] not in ("in", "emb", "front"):
                return None
            parts.extend(v[1] if v[0] == "front" else [v])
        if all(p[0] == "in" for p in parts) and len(parts) == 1:
            return parts[0]
        return ("front", parts)
    if node.op == "call_function" and node.target is operator.getitem:
        base, idx = sym.get(args[0]), args[1]
        if base is None or base[0] != "in" or not isinstance(idx, tuple) or len(idx) != 2:
            return None
        rows, c = idx
        if not (isinstance(rows, slice) and rows == slice(None, None, None)):
            return None
        cols = base[1]
        pick = (lambda i: i) if cols is None else (lambda i: cols[i])
        if isinstance(c, int):
            return ("col", pick(c)) if c >= 0 else None
        if isinstance(c, (list, tuple)) and c and all(isinstance(i, int) and i >= 0 for i in c):
            return ("in", [pick(i) for i in c])
        return None
    if node.op == "call_method" and node.target in ("long", "int") and len(args) == 1:
        v = sym.get(args[0])
        return ("icol", v[1]) if v is not None and v[0] == "col" else None
    if node.op == "call_module" and isinstance(mods.get(node.target), nn.Embedding) and len(args) == 1:
        v = sym.get(args[0])
        return ("emb", mods[node.target], v[1]) if v is not None and v[0] == "icol" else None
    return None


def fx_node_type():
    import torch.fx as fx
    return fx.Node


def _front_columns(v) -> Optional[List[FrontCol]]:
    parts = v[1] if v[0] == "front" else [v]
    out: List[FrontCol] = []
    for p in parts:
        if p[0] == "in":
            if p[1] is None:
                return None      # all raw columns inside a cat: width unknown at trace time
            out.extend(FrontCol(c) for c in p[1])
        elif p[0] == "emb":
            out.extend(FrontCol(p[2], p[1], j) for j in range(p[1].embedding_dim))
        else:
            return None
    return out
