"""ORACLE (test infrastructure only) -- CPU restatement of the reference's test harness.

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, as the checker.  Never imported by the product package.

Every function cites the reference lines it restates.  Pinned against fixtures that
``tests/golden/capture_golden.py`` recorded by running the reference's own
``network_test.TestNetwork`` / ``EpisodeDataloader`` / ``Classifier`` code in this
container (see tests/test_oracle_golden.py).
"""
from __future__ import annotations

import random as _random
from typing import Callable, Dict, List, Sequence

import numpy as np
import torch
from scipy.spatial.distance import cdist

# ------------------------------------------------------------------ episode sampling


def class_index(lines: Sequence[str]) -> Dict[str, List[str]]:
    """episode_novel_dataloader.py:25-32 -- class -> [video_info], first-appearance order."""
    d: Dict[str, List[str]] = {}
    for line in lines:
        line = line.strip("\n")
        d.setdefault(line.split("/")[0], []).append(line)
    return d


def sample_episode_plan(d: Dict[str, List[str]], n_way: int, k_shot: int, rnd=_random):
    """episode_novel_dataloader.py:34-70, RNG calls in the reference's order.

    Returns dict(query=video_info, query_y=int, support=[video_info], support_y=[int]).
    ``random.sample(dict.keys(), n)`` on Python 3.10 samples ``tuple(keys)``.
    """
    aim_class_names = rnd.sample(tuple(d.keys()), n_way)
    aim_query_name = rnd.sample(aim_class_names, 1)[0]
    support, support_y, query, query_y = [], [], None, None
    for class_name in aim_class_names:
        if class_name == aim_query_name:
            infos = rnd.sample(d[class_name], k_shot + 1)
            query = infos[0]
            query_y = aim_class_names.index(query.split("/")[0])
            infos = infos[1:]
        else:
            infos = rnd.sample(d[class_name], k_shot)
        for vi in infos:
            support.append(vi)
            support_y.append(aim_class_names.index(vi.split("/")[0]))
    return dict(query=query, query_y=query_y, support=support, support_y=support_y)


# ------------------------------------------------------------------ features


def video_embedding(model, video: torch.Tensor, L2: bool, n_frames: int | None = None) -> np.ndarray:
    """network_test.py:52-65 for ONE video: truncate, forward, F.normalize, np.mean(axis=0)."""
    if n_frames:
        video = video[0:n_frames]
    with torch.no_grad():
        feature, _ = model(video)
        if L2:
            feature = torch.nn.functional.normalize(feature, p=2, dim=1)
    return np.mean(feature.numpy(), axis=0)


def epoch_features(model, videos, L2: bool, frames=None) -> np.ndarray:
    """network_test.py:49-68 (generate_epoch_features)."""
    return np.array([video_embedding(model, videos[i], L2, frames[i] if frames else None)
                     for i in range(len(videos))])


def epoch_features_2(model, frames: torch.Tensor, L2: bool, batch_size: int = 96) -> np.ndarray:
    """network_test.py:70-99 (generate_epoch_features_2): per-frame features in chunks of 96."""
    out = []
    with torch.no_grad():
        for i in range(0, frames.shape[0], batch_size):
            f, _ = model(frames[i:i + batch_size])
            if L2:
                f = torch.nn.functional.normalize(f, p=2, dim=1)
            out.append(f.numpy())
    return np.concatenate(out, axis=0)


# ------------------------------------------------------------------ matching


def prototypes(support_feature: np.ndarray, support_y: np.ndarray):
    """classifier.py:9-40 -- per-label np.mean in first-appearance order."""
    groups: Dict[float, list] = {}
    for i in range(support_y.shape[0]):
        groups.setdefault(support_y[i], []).append(support_feature[i])
    ids = list(groups.keys())
    feats = np.array([np.mean(np.array(groups[c]), axis=0) for c in ids])
    return ids, feats


def protonet_predict(support_feature, support_y, query_feature, query_y):
    """classifier.py:43-90 -- f64 cdist -> f32 -> softmax(-d) -> argmax (position).

    The reference only supports one query (classifier.py:58 shadows query_feature).
    Returns (predicted_y int64[Q], distance f32[Q,P]).
    """
    _, protos = prototypes(support_feature, support_y)
    q = np.array([query_feature[i] for i in range(query_y.shape[0])])
    distance = torch.FloatTensor(cdist(q, protos, metric="euclidean"))
    prob = torch.nn.functional.softmax(-distance, dim=1)
    return np.argmax(prob.numpy(), axis=1), distance.numpy()


def cosine_predict(support_feature, query_feature):
    """classifier.py:117-120 -- sklearn cosine_similarity, argsort(-s)[:,0] (support index)."""
    from sklearn.metrics.pairwise import cosine_similarity

    s = cosine_similarity(query_feature, support_feature)
    return np.argsort(-s)[:, 0], s


def predict(kind: str, support_feature, support_y, query_feature, query_y):
    if kind == "protonet":
        return protonet_predict(support_feature, support_y, query_feature, query_y)[0]
    if kind == "cosine":
        return cosine_predict(support_feature, query_feature)[0]
    if kind == "SVM":  # classifier.py:109-111
        from sklearn.svm import SVC

        clf = SVC(C=10)
        clf.fit(support_feature, support_y)
        return clf.predict(query_feature)
    raise ValueError(kind)


# ------------------------------------------------------------------ drivers


def acc_lines(accs: Sequence[float]) -> List[str]:
    """network_test.py:162-167 -- running mean printed BEFORE the append (first is nan)."""
    import warnings

    lines, seen = [], []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i, a in enumerate(accs):
            lines.append(f"epoch: {i} acc: {a} avg_acc: {np.mean(seen)}")
            seen.append(a)
        lines.append(f"avg_acc: {np.mean(seen)}")
    return lines


def run_baseline(model, episodes: Sequence[dict], load_video: Callable, L2=True, kind="protonet"):
    """network_test.py:132-167 over pre-sampled episodes.

    ``load_video(video_info, support: bool) -> (tensor [n,3,H,W], n_frames)`` supplies
    frames; support videos are zero-padded to T with their real count (utils.py:215-258).
    Returns per-episode dict(support_feature, query_feature, pred, acc).
    """
    out = []
    for ep in episodes:
        sx, sf = zip(*[load_video(v, True) for v in ep["support"]])
        qx, _ = load_video(ep["query"], False)
        support_feature = epoch_features(model, list(sx), L2, list(sf))
        query_feature = epoch_features(model, [qx], L2)
        sy = np.array(ep["support_y"], dtype=np.float32)
        qy = np.array([ep["query_y"]], dtype=np.float32)
        pred = predict(kind, support_feature, sy, query_feature, qy)
        out.append(dict(support_feature=support_feature, query_feature=query_feature,
                        pred=pred, acc=float(np.mean(qy == pred))))
    return out


def temporal_smooth(distance: np.ndarray, lamda1=0.1, lamda2=1.0) -> np.ndarray:
    """network_test.py:103-117 + models.py:42-56 (PyTorch-1.x conv semantics).

    distance [S,G] f64 -> transpose -> f32 -> conv2d(kernel (1,3) = [l1,l2,l1],
    padding (0,1)) along S -> [S,G] f32.  Smoothing runs along the FLATTENED support
    segment axis (it crosses video boundaries), exactly as the reference does.
    """
    d = torch.FloatTensor(np.transpose(distance, (1, 0))).unsqueeze(0).unsqueeze(0)
    w = torch.FloatTensor([lamda1, lamda2, lamda1]).view(1, 1, 1, 3)
    y = torch.nn.functional.conv2d(d, w, padding=(0, 1))
    return np.transpose(y.view(y.shape[2], y.shape[3]).numpy(), (1, 0))


def aug_segment_episode(model, ep, load_video, gallery_seg_features, gallery_segments,
                        n_way, k_shot, T=16, seg_len=2, L2=True, kind="protonet"):
    """network_test.py:195-259 for one episode (data_aug='aug_seg_T').

    gallery_seg_features [G,D] f32 (D=2048), gallery_segments [G,seg_len,3,H,W].
    Reproduces the quirks: the 'probe' feature of support video i is flat segment i
    (:229), the smoothing crosses videos (:209), np.resize reshapes (:188,:204,:214).
    """
    num_segs = T // seg_len
    qx, _ = load_video(ep["query"], False)
    query_feature = epoch_features(model, [qx], L2)
    sx = torch.stack([load_video(v, True)[0] for v in ep["support"]])
    sy = np.array(ep["support_y"], dtype=np.float32)
    qy = np.array([ep["query_y"]], dtype=np.float32)
    H, W = sx.shape[-2:]
    support_segments = sx.view(-1, seg_len, 3, H, W)
    feats = epoch_features_2(model, sx.view(-1, 3, H, W), L2)
    D = feats.shape[1]
    seg_feats = np.mean(np.resize(feats, (n_way * k_shot * T // seg_len, seg_len, D)), axis=1)
    distance = temporal_smooth(cdist(seg_feats, gallery_seg_features, "euclidean"))
    pool_ids = np.resize(np.argsort(distance, axis=1)[:, :1], (n_way * k_shot, num_segs))
    support_segments = support_segments.view(n_way * k_shot, num_segs, seg_len, 3, H, W)
    aug_feats, aug_labels = [], []
    for i in range(pool_ids.shape[0]):
        aug_feats.append(seg_feats[i])
        aug_labels.append(sy[i])
        for s in range(num_segs):
            aug = support_segments[i].clone()
            aug[s] = gallery_segments[pool_ids[i][s]]
            aug_feats.append(video_embedding(model, aug.view(T, 3, H, W), L2))
            aug_labels.append(sy[i])
    aug_feats = np.array(aug_feats)
    aug_labels = np.array(aug_labels)
    pred = predict(kind, aug_feats, aug_labels, query_feature, qy)
    return dict(query_feature=query_feature, seg_features=seg_feats, pool_ids=pool_ids,
                aug_features=aug_feats, aug_labels=aug_labels, pred=pred,
                acc=float(np.mean(qy == pred)))
