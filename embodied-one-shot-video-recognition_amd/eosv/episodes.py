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


def shard(episodes: Sequence[dict], rank: int, world: int) -> List[dict]:
    """Episodes e with e % world == rank."""
    return [ep for i, ep in enumerate(episodes) if i % world == rank]
