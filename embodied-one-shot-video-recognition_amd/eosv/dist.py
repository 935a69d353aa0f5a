"""Episode data-parallelism over ranks.

Episodes are independent, so rank r runs episodes e with e % world == r (the plans
are sampled once, in the reference's RNG order, identically on every rank).  The
only collective is ONE all-gather of per-episode int64 (episode, prediction) pairs
after the run (RCCL over xGMI with the "nccl" backend, gloo on CPU), from which
every rank rebuilds the predictions in global episode order; the mean of 0/1
accuracies is then exact, so the result equals the single-GPU run bit for bit.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch


def world():
    d = torch.distributed
    if d.is_available() and d.is_initialized():
        return d, d.get_rank(), d.get_world_size()
    return None, 0, 1


def shard_indices(n: int, rank: int, n_ranks: int):
    return list(range(rank, n, n_ranks))


def _coll_device(d):
    if d.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_predictions(local_idx: Sequence[int], local_pred: Sequence[int], n_total: int) -> np.ndarray:
    """All ranks' (episode, pred) -> int64 [n_total] predictions in global order (all ranks)."""
    d, rank, n_ranks = world()
    preds = np.full(n_total, -1, np.int64)
    if d is None:
        preds[np.asarray(local_idx, np.int64)] = np.asarray(local_pred, np.int64)
        return preds
    dev = _coll_device(d)
    n_max = (n_total + n_ranks - 1) // n_ranks
    buf = torch.full((n_max, 2), -1, dtype=torch.int64, device=dev)
    k = len(local_idx)
    if k:
        buf[:k, 0] = torch.as_tensor(np.asarray(local_idx, np.int64), device=dev)
        buf[:k, 1] = torch.as_tensor(np.asarray(local_pred, np.int64), device=dev)
    parts = [torch.empty_like(buf) for _ in range(n_ranks)]
    d.all_gather(parts, buf)
    allb = torch.cat(parts).cpu().numpy()
    allb = allb[allb[:, 0] >= 0]
    preds[allb[:, 0]] = allb[:, 1]
    return preds


def all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    """Every rank's rows of ``x`` ([n_r, ...], any n_r), concatenated in rank order, on x's device.

    Used by the config-3 driver to shard the gallery forward: rank r computes a
    contiguous block of gallery videos and one all-gather (RCCL over xGMI, or gloo through the
    host) rebuilds the full per-frame feature table on every rank.  The backbone computes every
    frame independently of its batch, so the table is bit-identical to the unsharded one."""
    d, _, n_ranks = world()
    if d is None or n_ranks == 1:
        return x
    dev = _coll_device(d)
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(n_ranks)]
    d.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    m = max(ns)
    buf = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=dev)
    buf[:x.shape[0]] = x.to(dev)
    parts = [torch.empty_like(buf) for _ in range(n_ranks)]
    d.all_gather(parts, buf)
    return torch.cat([p[:k] for p, k in zip(parts, ns)]).to(x.device)


def block_range(n: int, rank: int, n_ranks: int):
    """Contiguous block [lo, hi) of n items for rank (the first n % n_ranks ranks take one more)."""
    q, r = divmod(n, n_ranks)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (rank < r)


def max_over_ranks(x: float) -> float:
    d, _, _ = world()
    if d is None:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_coll_device(d))
    d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: int) -> int:
    d, _, _ = world()
    if d is None:
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64, device=_coll_device(d))
    d.all_reduce(t)
    return int(t.item())


def gather_values(x: float):
    """[x of rank 0, x of rank 1, ...] on every rank (one all-gather of an f64 scalar)."""
    d, _, n_ranks = world()
    if d is None:
        return [float(x)]
    dev = _coll_device(d)
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    parts = [torch.empty_like(t) for _ in range(n_ranks)]
    d.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def describe():
    """What the process group itself reports: backend name and world size (None when single-process)."""
    d, _, _ = world()
    if d is None:
        return {"backend": None, "world_size_reported_by_backend": 1}
    return {"backend": d.get_backend(), "world_size_reported_by_backend": d.get_world_size()}


def episode_accs(preds: np.ndarray, query_y: Sequence[int]):
    """np.mean(query_y == predicted_y) per episode (network_test.py:159): 0.0 / 1.0."""
    return [np.mean(np.array([query_y[e]], np.float32) == preds[e]) for e in range(len(preds))]
