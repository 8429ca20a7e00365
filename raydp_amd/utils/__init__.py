"""General helpers of the public ``raydp.utils`` surface.

Parity: ``python/raydp/utils.py`` of the reference (``parse_memory_size`` :125-146,
``random_split`` :67-83, ``df_type_check``/``convert_to_spark``/``_df_helper`` :86-122,
``divide_blocks`` :149-222, ``get_node_address`` :34-58, ``register_exit_handler`` :61-64).

The DataFrame types accepted here are this framework's own Arrow-native Spark-compatible
``DataFrame`` (``raydp_amd.spark.DataFrame``) and its pandas-on-Spark subset
(``raydp_amd.spark.pandas.DataFrame``); there is no PySpark in this environment.
"""
import atexit
import math
import os
import re
import signal
import socket
from typing import Dict, List, Tuple

import numpy as np

MEMORY_SIZE_UNITS = {"K": 2 ** 10, "M": 2 ** 20, "G": 2 ** 30, "T": 2 ** 40}

BLOCK_SIZE_BIT = 32

__all__ = [
    "parse_memory_size", "random_split", "divide_blocks", "df_type_check",
    "convert_to_spark", "get_node_address", "register_exit_handler", "get_node_ip_address",
    "MEMORY_SIZE_UNITS",
]


# runtime "memory" resources are accounted in bytes (Ray >= 2 semantics)
MEMORY_RESOURCE_UNIT_BYTES = 1

def get_node_ip_address() -> str:
    """IP of this node as seen by peers; loopback when the host name does not resolve."""
    env = os.environ.get("RAYDP_NODE_IP")
    if env:
        return env
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect(("10.255.255.255", 1))
            ip = s.getsockname()[0]
        finally:
            s.close()
        return ip
    except OSError:
        return "127.0.0.1"


def get_node_address() -> str:
    """Address of the local runtime node (reference scans psutil for ``--node-ip-address``)."""
    from raydp_amd import runtime
    if runtime.is_initialized():
        return runtime.get_runtime_context().node_ip
    return get_node_ip_address()


def register_exit_handler(func):
    atexit.register(func)
    signal.signal(signal.SIGTERM, func)
    signal.signal(signal.SIGINT, func)


def random_split(df, weights, seed=None):
    """Random split a DataFrame (or pandas-on-Spark DataFrame) into parts.

    Weights are normalised when they do not sum to 1.0. Splitting is a per-row Bernoulli
    draw keyed by ``(seed, partition)``; it is deterministic for a seed but not
    bit-identical to Spark's XORShift sampler.
    """
    df, is_spark_df = convert_to_spark(df)
    splits = df.randomSplit(weights, seed)
    if is_spark_df:
        return splits
    from raydp_amd.spark import pandas as ps
    return [ps.DataFrame(split) for split in splits]


def _df_helper(df, spark_callback, spark_pandas_callback):
    from raydp_amd.spark.dataframe import DataFrame
    from raydp_amd.spark import pandas as ps
    if isinstance(df, DataFrame):
        return spark_callback(df)
    if isinstance(df, ps.DataFrame):
        return spark_pandas_callback(df)
    raise Exception(f"The type: {type(df)} is not supported, only support "
                    "raydp DataFrame and pandas-on-Spark DataFrame")


def df_type_check(df):
    """True for a Spark-style or pandas-on-Spark DataFrame; raises otherwise."""
    return _df_helper(df, lambda d: True, lambda d: True)


def convert_to_spark(df):
    """Return ``(spark_df, is_spark_df)``; pandas-on-Spark frames are converted."""
    return _df_helper(df, lambda d: (d, True), lambda d: (d.to_spark(), False))


_SIZE_RE = re.compile(r"^\s*([0-9]*\.?[0-9]+)\s*([KMGT]?)(?:I?B)?\s*$", re.IGNORECASE)


def parse_memory_size(memory_size) -> int:
    """Bytes of a human readable size: "10", "10K", "10 kb", "1.5g", "2 GiB" (powers of 1024,
    reference ``python/raydp/utils.py:125-146``)."""
    if isinstance(memory_size, (int, np.integer)):
        return int(memory_size)
    m = _SIZE_RE.match(str(memory_size))
    if m is None:
        raise ValueError(f"cannot parse memory size {memory_size!r}")
    number, unit = m.group(1), m.group(2).upper()
    scale = MEMORY_SIZE_UNITS.get(unit, 1)
    return int(float(number) * scale) if "." in number else int(number) * scale


def divide_blocks(blocks: List[int], world_size: int, shuffle: bool = False,
                  shuffle_seed: int = None) -> Dict[int, List[Tuple[int, int]]]:
    """Assign blocks to ranks so that every rank gets exactly the same number of samples.

    Returns ``{rank: [(block_index, num_samples_taken), ...]}``. Blocks are dealt round-robin
    (after an optional seeded shuffle); a rank that is short pads with randomly chosen
    blocks, a rank that overflows truncates its last block.
    """
    if len(blocks) < world_size:
        raise Exception("do not have enough blocks to divide")
    rng = np.random.RandomState(shuffle_seed if shuffle_seed else 0)
    per_rank_blocks = int(math.ceil(len(blocks) / world_size))
    per_rank_samples = int(math.ceil(sum(blocks) / world_size))
    total = per_rank_blocks * world_size
    order = list(range(len(blocks)))
    order += order[: total - len(order)]
    if shuffle:
        rng.shuffle(order)

    results = {}
    for rank in range(world_size):
        chosen: List[Tuple[int, int]] = []
        have = 0

        def take(idx, have):
            room = per_rank_samples - have
            n = min(blocks[idx], room)
            chosen.append((idx, n))
            return have + n

        for idx in order[rank:total:world_size]:
            have = take(idx, have)
            if have == per_rank_samples:
                break
        while have < per_rank_samples:
            have = take(int(rng.choice(order)), have)
        results[rank] = chosen
    return results


def partition_cpus(local_rank: int, local_world: int, min_per_rank: int = 2):
    """The CPU slice of one local rank when ``local_world`` ranks share a node: contiguous,
    equal slices of the cores this process may use (rank r -> the r-th slice, so with the usual
    MI355X layout of GPUs 0-3 on socket 0 and 4-7 on socket 1 a rank's host work stays on its
    GPU's socket). None when the node has fewer than ``min_per_rank`` cores per rank (then
    overlapping slices would only add contention) or there is nothing to split."""
    import os
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    if local_world <= 1 or len(cpus) < min_per_rank * local_world:
        return None
    per = len(cpus) // local_world
    return cpus[local_rank * per:(local_rank + 1) * per]


def pin_to_rank_slice(local_rank: int, local_world: int, min_per_rank: int = 2):
    """Confine this process -- and every process it starts afterwards (the runtime supervisor,
    executor and worker actors inherit it) -- to its rank's CPU slice. Returns the slice or None."""
    import os
    cpus = partition_cpus(local_rank, local_world, min_per_rank)
    if cpus:
        try:
            os.sched_setaffinity(0, cpus)
        except OSError:
            return None
    return cpus
