"""Episode planning in the reference's RNG order (episode_novel_dataloader.py:19-80).

The reference rebuilds a class -> [video_info] dict from the split list on every
call and draws, from the GLOBAL ``random`` module:
    random.sample(dict.keys(), n_way)          # :35 (Python 3.10: samples tuple(keys))
    random.sample(aim_class_names, 1)[0]       # :37
    random.sample(videos, k_shot + 1 | k_shot) # :48 / :58, class by class
Support label = index of the class in the sampled order (:53, :68); supports are
appended class by class; exactly one query per episode.  Plans are sampled on the
host up front (cheap) so that episodes can be batched and sharded over GPUs
without changing which videos each episode uses.
"""
from __future__ import annotations

import os
import random as _random
from typing import Dict, List, Sequence

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LISTS = {"train": "sources/data/train.list", "val": "sources/data/val.list", "test": "sources/data/test.list"}


def read_list(mode: str = "test", root: str = PKG_ROOT) -> List[str]:
    with open(os.path.join(root, LISTS[mode])) as f:
        return f.readlines()


def class_index(lines: Sequence[str]) -> Dict[str, List[str]]:
    d: Dict[str, List[str]] = {}
    for line in lines:
        line = line.strip("\n")
        d.setdefault(line.split("/")[0], []).append(line)
    return d


def sample_episode(index: Dict[str, List[str]], n_way: int, k_shot: int, rnd=_random) -> dict:
    names = rnd.sample(tuple(index.keys()), n_way)
    query_name = rnd.sample(names, 1)[0]
    support, support_y, query, query_y = [], [], None, None
    for cname in names:
        if cname == query_name:
            infos = rnd.sample(index[cname], k_shot + 1)
            query, infos = infos[0], infos[1:]
            query_y = names.index(query.split("/")[0])
        else:
            infos = rnd.sample(index[cname], k_shot)
        for vi in infos:
            support.append(vi)
            support_y.append(names.index(vi.split("/")[0]))
    return dict(support=support, support_y=support_y, query=query, query_y=query_y)


def sample_episodes(n: int, n_way: int = 5, k_shot: int = 1, mode: str = "test", seed=None,
                    rnd=None, lines=None) -> List[dict]:
    """n episode plans.  ``seed`` -> a private Random; else ``rnd`` or the global module."""
    if rnd is None:
        rnd = _random.Random(seed) if seed is not None else _random
    index = class_index(lines if lines is not None else read_list(mode))
    return [sample_episode(index, n_way, k_shot, rnd) for _ in range(n)]


def plan_episodes(n: int, n_way: int = 5, k_shot: int = 1, mode: str = "test", seed: int = 0,
                  lines=None) -> List[dict]:
    """The native plan service (csrc/plan.hip ``eosv_plan_episodes``): the same plans as
    ``sample_episodes(n, n_way, k_shot, mode, seed=seed)``, drawn in C++ from a restated
    CPython MT19937 without a per-episode dict rebuild.  ``seed``: int in [0, 2**64)."""
    import ctypes

    import numpy as np

    from . import _lib

    index = class_index(lines if lines is not None else read_list(mode))
    names = list(index.keys())
    sizes = np.array([len(index[c]) for c in names], dtype=np.int32)
    classes = np.zeros((max(n, 1), n_way), dtype=np.int32)
    query = np.zeros((max(n, 1), 2), dtype=np.int32)
    support = np.zeros((max(n, 1), n_way, max(k_shot, 1)), dtype=np.int32)
    if not 0 <= int(seed) < 2 ** 64:
        raise ValueError("plan_episodes: seed must be in [0, 2**64)")
    _lib.check(_lib.lib().eosv_plan_episodes(sizes.ctypes.data, len(names), n_way, k_shot, ctypes.c_uint64(int(seed)),
                                             n, classes.ctypes.data, query.ctypes.data, support.ctypes.data),
               "eosv_plan_episodes")
    plans = []
    for e in range(n):
        cls = [names[c] for c in classes[e]]
        qpos = int(query[e, 0])
        sup, sup_y = [], []
        for i, c in enumerate(cls):
            for s in range(k_shot):
                sup.append(index[c][support[e, i, s]])
                sup_y.append(i)
        plans.append(dict(support=sup, support_y=sup_y, query=index[cls[qpos]][query[e, 1]], query_y=qpos))
    return plans


def shard(episodes: Sequence[dict], rank: int, world: int) -> List[dict]:
    """Episodes e with e % world == rank."""
    return [ep for i, ep in enumerate(episodes) if i % world == rank]
