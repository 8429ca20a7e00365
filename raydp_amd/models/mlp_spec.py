"""Recognise fusable MLPs in user ``nn.Module``s (torch.fx pattern match).

A model qualifies for the fused HIP trainer when its traced graph is a single chain of
``Linear`` layers, each hidden one followed by an optional activation (ReLU / identity) and an
optional ``BatchNorm1d`` in either order, ending in a bare ``Linear``. That covers the
reference's ``NYC_Model`` (``examples/pytorch_nyctaxi.py:69-92``: Linear→ReLU→BN ×4 →
Linear), the ``LinearModel`` of ``tests/test_torch.py`` and DLRM-style MLP towers.
Anything else (dropout, residuals, embeddings, custom ops) returns ``None`` and the generic
device-resident PyTorch loop is used instead.
"""
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
class MlpSpec:
    layers: List[LayerSpec] = field(default_factory=list)

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
        spec = MlpSpec()
        for lin, act, bn, bn_name in recipe:
            spec.layers.append(LayerSpec(linear=model.get_submodule(lin), act=act, bn=bn,
                                         bn_module=model.get_submodule(bn_name) if bn_name else None))
        return spec
    spec = _trace_spec(model)
    if key is not None:
        if len(_SPEC_CACHE) > 256:
            _SPEC_CACHE.clear()
        if spec is None:
            _SPEC_CACHE[key] = None
        else:
            names = {id(m): n for n, m in model.named_modules()}
            _SPEC_CACHE[key] = [(names[id(ly.linear)], ly.act, ly.bn,
                                 names[id(ly.bn_module)] if ly.bn_module is not None else None)
                                for ly in spec.layers]
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
    saw_act_after_bn = False
    for node in gm.graph.nodes:
        if node.op == "placeholder":
            if placeholder is not None:
                return None  # multi-input models are not MLP chains
            placeholder = node
            prev_node = node
            continue
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
    return spec
