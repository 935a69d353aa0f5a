"""Drop-in for the reference's ``network_test.py`` (TestNetwork, lines 23-267), on MI355X.

Same constructor, methods, printed lines and result-file format as the reference.
What changes is the execution strategy:

* ``test_network_baseline`` pre-samples every episode plan with the global RNG in
  the reference's order (test/val loading draws nothing from the RNG, so the plans
  are the reference's), then runs batches of ``episodes_per_batch`` episodes as ONE
  frame table in HBM: one backbone call, one clip-embed launch, one match launch.
  Only int64 predictions come back to the host.
* ``test_network_aug_segment`` computes the gallery segment features once, then per
  batch of episodes: support/query features in one forward, gallery matching
  (f64 cdist + temporal smoothing + argmin) on the GPU, the 40 augmented videos per
  episode gathered on the device and embedded in one forward, protonet matching.
* With ``torch.distributed`` initialised, episode e runs on rank e % world and the
  per-episode (prediction, correct) pairs are all-gathered; rank 0 writes the file.

Synthetic frames (no dataset offline) are generated directly in HBM; real JPEG
frame directories are decoded on the host (eosv.frames).
"""
import copy
import warnings

import os

import numpy as np
import torch

import utils
from classifier import Classifier
from episode_novel_dataloader import EpisodeDataloader
from eosv import dist as _dist_mod, engine as _engine, frames as _frames, synth as _synth
from models import TemporalLayer, model_resnet18, model_resnet50, model_resnet101
import generate_augmented_datasets as _gad

_MODELS = {'resnet18': model_resnet18, 'resnet50': model_resnet50, 'resnet101': model_resnet101}


def _dist():
    return _dist_mod.world()


class TestNetwork():
    #: episodes per device batch in the batched drivers
    episodes_per_batch = 64

    def __init__(self, test_result_txt, resnet_model='resnet50', classifier='protonet', L2=True,
                 num_classes=utils.num_classes_train, mode='test'):
        self.test_result_txt = test_result_txt
        self.resnet_model = resnet_model
        self.classifier = classifier
        self.L2 = L2
        self.num_classes = num_classes
        self.mode = mode
        if resnet_model not in _MODELS:
            raise ValueError(f"resnet_model must be one of {list(_MODELS)}")
        self.mymodel = _MODELS[resnet_model](num_classes=self.num_classes)
        self.mymodel.eval()
        self.mymodel.cuda()
        print('model loaded.')
        self.myEpisodeDataloader = EpisodeDataloader(mode=self.mode)
        self.myClassifier = Classifier(classifier=self.classifier)

    # ------------------------------------------------------------------ features
    def _backbone(self, H, W):
        return self.mymodel.native(H, W)

    def _features(self, frames):
        """frames [F,3,H,W] (host or device) -> per-frame features [F,D] on the device."""
        if not frames.is_cuda:
            frames = frames.cuda()
        frames = frames.float().contiguous()
        return self._backbone(frames.shape[2], frames.shape[3]).forward(frames)

    def generate_epoch_features(self, videos, L2=False, support_x_frames=None):
        """network_test.py:49-68: per-video mean of (L2-normalised) frame features -> np [V,D].

        All videos go through ONE backbone call; truncation to support_x_frames[i]
        (:54-55) becomes the clip length."""
        V = videos.shape[0]
        counts = [int(support_x_frames[i]) if support_x_frames else int(videos[i].shape[0]) for i in range(V)]
        frames = torch.cat([videos[i][0:counts[i]] for i in range(V)])
        feat = self._features(frames)
        offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
        dev = feat.device
        emb = _engine.clip_embed(feat, torch.from_numpy(offs).to(dev),
                                 torch.from_numpy(np.array(counts, np.int32)).to(dev), bool(L2))
        return emb.cpu().numpy()

    def generate_epoch_features_2(self, videos, L2=False):
        """network_test.py:70-99: per-frame (L2-normalised) features -> np [F,D]."""
        feat = self._features(videos)
        if L2:
            n = feat.shape[0]
            dev = feat.device
            feat = _engine.clip_embed(feat, torch.arange(n, dtype=torch.int32, device=dev),
                                      torch.ones(n, dtype=torch.int32, device=dev), True)
        return feat.cpu().numpy()

    def temporal_convolution_flating_layer(self, distance):
        """network_test.py:103-117: [S,G] -> smoothed along S (TemporalLayer on the transpose)."""
        d = torch.from_numpy(np.ascontiguousarray(np.transpose(np.asarray(distance), (1, 0)), dtype=np.float32))
        y = TemporalLayer()(d.cuda())
        return np.transpose(y.cpu().numpy(), (1, 0))

    def video_segment_augmentation(self, video_probe_seg, seg_id, gallery_seg, data_aug=None):
        """network_test.py:119-129 (host numpy, as in the reference)."""
        aug_video = copy.deepcopy(video_probe_seg)
        if data_aug == 'aug_image_gaussian':
            aug_video[seg_id] = aug_video[seg_id] + np.random.normal(0, 0.3, (utils.seg_len, 3, 224, 224))
        elif data_aug == 'aug_frame_gaussian':
            pass
        else:
            aug_video[seg_id] = gallery_seg
        return np.resize(aug_video, (utils.VIDEO_FRAMES, 3, 224, 224))

    # ------------------------------------------------------------------ frame tables
    def _clip_frames(self, clips, H, W, dev):
        """clips: list of (video_info, [frame ids], pad_to). Frame id 0 = a zero frame.
        Returns frames [F,3,H,W] f32 on the device (synthetic: generated in HBM)."""
        src = utils.frame_source()
        if src.synthetic:
            rows = []
            for vi, ids, pad_to in clips:
                cls = vi.split('/')[0]
                cs, vs, crc = _synth.class_seed(cls), _synth.video_seed(vi), _synth.crc32(vi)
                for f in ids:
                    rows.append((cs, vs, _synth.mix64_int(((crc << 20) + f) ^ _synth.TAG_NOISE), f))
                rows += [(0, 0, 0, 0)] * (pad_to - len(ids))
            return _engine.synth_frames(np.array(rows, np.uint64).reshape(-1, 4), H, W, dev)
        # real frames: JPEG decode on the host, crop + normalise on the GPU (eosv/frames.py)
        out = []
        for vi, ids, pad_to in clips:
            v = src.frames_tensor(vi, ids, 'test').to(dev)
            if pad_to > len(ids):
                v = torch.cat([v, torch.zeros(pad_to - len(ids), 3, H, W, device=v.device)])
            out.append(v)
        return torch.cat(out)

    def _ids(self, vi, mode):
        n_all = utils.frame_source().frame_count(vi)
        return _frames.clip_frame_ids(n_all, utils.VIDEO_FRAMES, mode)

    # ------------------------------------------------------------------ drivers
    def _load(self, pre_model):
        if pre_model:
            self.mymodel.load_state_dict(torch.load(pre_model, map_location='cpu', weights_only=True))
            print(pre_model, 'loaded.')
        self.mymodel.eval()

    def _write_results(self, accs):
        """network_test.py:161-167: running mean printed BEFORE the append."""
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            s = 0.0
            for epoch, acc in enumerate(accs):
                avg = np.mean([]) if epoch == 0 else np.float64(s / epoch)
                print('epoch:', epoch, 'acc:', acc, 'avg_acc:', avg)
                print('epoch:', epoch, 'acc:', acc, 'avg_acc:', avg, file=self.acc_file)
                s += float(acc)
            avg_acc = np.mean([]) if not accs else np.float64(s / len(accs))
        print('avg_acc:', avg_acc)
        print('avg_acc:', avg_acc, file=self.acc_file)
        self.acc_file.flush()
        return avg_acc

    def _gather(self, local_idx, local_pred, n_total, qys):
        """(episode, pred) from every rank -> accs in global episode order (eosv.dist)."""
        preds = _dist_mod.gather_predictions(local_idx, local_pred, n_total)
        return _dist_mod.episode_accs(preds, qys), preds

    def test_network_baseline(self, pre_model=None):
        """network_test.py:132-167, batched over episodes (and ranks)."""
        self._load(pre_model)
        d, rank, world = _dist()
        self.acc_file = open(self.test_result_txt, 'w') if rank == 0 else None
        n = utils.EPISODE_NUMS[self.mode]
        if self.mode == 'train':  # train-mode loading consumes the RNG: keep the per-episode loop
            return self._baseline_per_episode(n)
        plans = [self.myEpisodeDataloader.get_episode_plan() for _ in range(n)]
        mine = list(range(rank, n, world))
        preds = []
        for b0 in range(0, len(mine), self.episodes_per_batch):
            preds += self._baseline_batch([plans[e] for e in mine[b0:b0 + self.episodes_per_batch]])
        accs, all_preds = self._gather(mine, preds, n, [p['query_y'] for p in plans])
        self.last_accs, self.last_preds = accs, all_preds
        if rank == 0:
            return self._write_results(accs)

    def _baseline_batch(self, plans):
        H, W = utils.IMG_crop_size
        dev = torch.device('cuda', torch.cuda.current_device())
        clips, sup_off, slots, nproto = [], [0], [], []
        for p in plans:
            seen = {}
            for vi, y in zip(p['support'], p['support_y']):
                ids = self._ids(vi, self.mode)
                clips.append((vi, ids, len(ids)))
                slots.append(seen.setdefault(int(y), len(seen)))
            sup_off.append(sup_off[-1] + len(p['support']))
            nproto.append(len(seen))
        for p in plans:
            ids = self._ids(p['query'], 'test')
            clips.append((p['query'], ids, len(ids)))
        counts = np.array([len(c[1]) for c in clips], np.int32)
        offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
        frames = self._clip_frames(clips, H, W, dev)
        feat = self._features(frames)
        t = lambda a: torch.from_numpy(np.asarray(a, np.int32)).to(dev)  # noqa: E731
        emb = _engine.clip_embed(feat, t(offs), t(counts), bool(self.L2))
        ns = sup_off[-1]
        if self.classifier not in ('protonet', 'cosine'):  # SVM (host sklearn), KNN / unknown: raise as the reference
            return self._host_classify(emb, sup_off, [np.asarray(p['support_y'], np.float32) for p in plans],
                                       [p['query_y'] for p in plans])
        pred, _ = _engine.match(emb[ns:].contiguous(), emb[:ns].contiguous(), t(sup_off), t(slots), t(nproto),
                                self.classifier)
        debug = getattr(self, 'debug', None)
        if debug is not None:  # tests: per-batch clip embeddings (supports, then queries)
            debug.setdefault('batches', []).append(dict(sup=emb[:ns], q=emb[ns:], sup_off=sup_off, pred=pred))
        return pred.cpu().tolist()

    def _host_classify(self, emb, sup_off, sup_y, query_y):
        """Classifier.predict per episode on the host (classifier.py:98-123) for the classifiers
        the match kernel does not run: episode e's supports are rows sup_off[e]..sup_off[e+1]
        of `emb`, its query row sup_off[-1] + e."""
        emb = emb.cpu().numpy()
        ns = sup_off[-1]
        preds = []
        for e in range(len(sup_y)):
            res = {'support_feature': emb[sup_off[e]:sup_off[e + 1]], 'support_y': sup_y[e],
                   'query_feature': emb[ns + e:ns + e + 1], 'query_y': np.array([query_y[e]], np.float32)}
            preds.append(int(np.asarray(self.myClassifier.predict(res)).reshape(-1)[0]))
        return preds

    def _baseline_per_episode(self, n):
        accs = []
        for _ in range(n):
            data = self.myEpisodeDataloader.get_episode()
            sf = self.generate_epoch_features(data['support_x'], self.L2, data['support_x_frames'])
            qf = self.generate_epoch_features(data['query_x'], self.L2)
            res = {'support_feature': sf, 'support_y': data['support_y'].numpy(),
                   'query_feature': qf, 'query_y': data['query_y'].numpy()}
            accs.append(np.mean(res['query_y'] == self.myClassifier.predict(res)))
        self.last_accs = accs
        return self._write_results(accs)

    # ------------------------------------------------------------------ config 3
    def gallery_features(self):
        """Gallery segment features [G*T/seg_len, D] on the device (network_test.py:184-189).

        Also keeps the raw (pre-L2) per-frame gallery features, np.resize'd like the segment
        features: the augmented videos of aug_seg_T are assembled from gallery and support
        FRAMES, and the backbone is a per-frame 2D CNN whose kernels compute every frame with
        the same instruction sequence wherever it sits in a batch, so their features are
        gathered instead of re-running the backbone on the assembled frames (bit-identical;
        EOSV_AUG_REFORWARD=1 re-runs it, as the reference does at network_test.py:210-248)."""
        H, W = utils.IMG_crop_size
        T, sl = utils.VIDEO_FRAMES, utils.seg_len
        dev = torch.device('cuda', torch.cuda.current_device())
        infos = _gad.gallery_video_infos()
        clips_all = []
        for vi in infos:  # every rank checks every video, so a bad list fails on all ranks alike
            ids = self._ids(vi, 'test')
            if len(ids) != T:
                raise ValueError(f"gallery video {vi} has {len(ids)} < {T} frames "
                                 "(the reference's torch.stack fails on it too)")
            clips_all.append((vi, ids, T))
        feats, raws = [], []
        self._gallery_frames = [] if self._aug_reforward() else None
        # multi-rank: each rank forwards a contiguous block of the gallery videos and one
        # all-gather rebuilds the table; the re-forward mode keeps every frame local
        _, rank, world = _dist()
        lo, hi = (0, len(clips_all)) if self._gallery_frames is not None else _dist_mod.block_range(
            len(clips_all), rank, world)
        for g0 in range(lo, hi, 64):
            clips = clips_all[g0:min(g0 + 64, hi)]
            fr = self._clip_frames(clips, H, W, dev)
            if self._gallery_frames is not None:
                self._gallery_frames.append(fr)
            f = self._features(fr)
            raws.append(f)
            if self.L2:
                n = f.shape[0]
                f = _engine.clip_embed(f, torch.arange(n, dtype=torch.int32, device=dev),
                                       torch.ones(n, dtype=torch.int32, device=dev), True)
            feats.append(f)
        D = self._backbone(H, W).D
        feat = torch.cat(feats) if feats else torch.empty((0, D), device=dev)
        raw = torch.cat(raws) if raws else torch.empty((0, D), device=dev)
        if self._gallery_frames is None:
            feat, raw = _dist_mod.all_gather_rows(feat), _dist_mod.all_gather_rows(raw)
        if feat.shape[1] != 2048:
            raise ValueError("test_network_aug_segment needs a 2048-d backbone (resnet50/101): the reference "
                             "np.resize's features to 2048 (network_test.py:188,204)")
        n_seg = 640 * T // sl
        if feat.shape[0] != n_seg * sl:  # np.resize semantics: repeat/truncate the flat array
            reps = torch.arange(n_seg * sl, device=dev) % feat.shape[0]
            feat = feat[reps].contiguous()
            raw = raw[reps].contiguous()
        self._gallery_raw = raw
        if self._gallery_frames is not None:
            self._gallery_frames = torch.cat(self._gallery_frames)
        return _engine.segment_mean(feat, sl)

    @staticmethod
    def _aug_reforward():
        return os.environ.get("EOSV_AUG_REFORWARD", "0") == "1"

    def test_network_aug_segment(self, pre_model=None, data_aug='aug_seg_T'):
        """network_test.py:170-267, batched on the device."""
        self._load(pre_model)
        d, rank, world = _dist()
        self.acc_file = open(self.test_result_txt, 'w') if rank == 0 else None
        print("preaparing gallery segments.")
        if data_aug != 'aug_seg_T':
            print('data_aug error.')
            return 0
        gal = self.gallery_features()
        n = utils.EPISODE_NUMS[self.mode]
        plans = [self.myEpisodeDataloader.get_episode_plan() for _ in range(n)]
        mine = list(range(rank, n, world))
        preds = []
        B = max(1, self.episodes_per_batch // 8)
        for b0 in range(0, len(mine), B):
            preds += self._aug_batch([plans[e] for e in mine[b0:b0 + B]], gal, getattr(self, 'debug', None))
        accs, _ = self._gather(mine, preds, n, [p['query_y'] for p in plans])
        self.last_accs = accs
        if rank == 0:
            return self._write_results(accs)

    def _aug_batch(self, plans, gal, debug=None):
        H, W = utils.IMG_crop_size
        T, sl = utils.VIDEO_FRAMES, utils.seg_len
        ns_v = T // sl
        dev = torch.device('cuda', torch.cuda.current_device())
        E = len(plans)
        nk = len(plans[0]['support'])
        clips = []
        for p in plans:  # supports: zero padded to T, no truncation (network_test.py:201-203)
            for vi in p['support']:
                clips.append((vi, self._ids(vi, self.mode), T))
        for p in plans:
            ids = self._ids(p['query'], 'test')
            clips.append((p['query'], ids, len(ids)))
        frames = self._clip_frames(clips, H, W, dev)
        feat = self._features(frames)
        n_sup_frames = E * nk * T
        q_counts = np.array([len(c[1]) for c in clips[E * nk:]], np.int32)
        q_offs = (n_sup_frames + np.concatenate([[0], np.cumsum(q_counts)[:-1]])).astype(np.int32)
        t = lambda a: torch.from_numpy(np.asarray(a, np.int32)).to(dev)  # noqa: E731
        q_emb = _engine.clip_embed(feat, t(q_offs), t(q_counts), bool(self.L2))
        sf = feat[:n_sup_frames]
        if self.L2:
            sf = _engine.clip_embed(sf.contiguous(), torch.arange(n_sup_frames, dtype=torch.int32, device=dev),
                                    torch.ones(n_sup_frames, dtype=torch.int32, device=dev), True)
        seg = _engine.segment_mean(sf.contiguous(), sl)  # [E*nk*ns_v, D]
        S = nk * ns_v
        # every episode's segments against the gallery in one launch (per-episode smoothing)
        pool, _ = _engine.segment_match_episodes(seg.contiguous(), E, gal, utils.lamda1, utils.lamda2)
        pool = pool.view(E, nk, ns_v)  # np.resize(pool_ids, (n*k, num_segs))
        # augmented videos: support video i with segment s <- gallery segment pool[e,i,s]
        f = torch.arange(T, device=dev)
        seg_of = f // sl
        s_idx = torch.arange(ns_v, device=dev)
        sup_rows = (torch.arange(E * nk, device=dev).view(E, nk, 1, 1) * T + f.view(1, 1, 1, T))
        gal_rows = (pool.view(E, nk, ns_v, 1) * sl + (f % sl).view(1, 1, 1, T))
        use_gal = (seg_of.view(1, 1, 1, T) == s_idx.view(1, 1, ns_v, 1))
        n_gal = self._gallery_raw.shape[0]
        rows = torch.where(use_gal, gal_rows, n_gal + sup_rows.expand(E, nk, ns_v, T)).reshape(-1)
        if self._gallery_frames is not None:  # the reference's way: forward the assembled frames
            src = torch.cat([self._gallery_frames, frames[:n_sup_frames]])
            aug_feat = self._features(src.index_select(0, rows))
        else:  # per-frame CNN: gather the frames' features (see gallery_features)
            aug_feat = torch.cat([self._gallery_raw, feat[:n_sup_frames]]).index_select(0, rows).contiguous()
        n_aug = E * nk * ns_v
        aug_emb = _engine.clip_embed(aug_feat, torch.arange(n_aug, dtype=torch.int32, device=dev) * T,
                                     torch.full((n_aug,), T, dtype=torch.int32, device=dev), bool(self.L2))
        # support set per episode: [probe_i (= flat segment i, :229), aug_i0..aug_i7] for i < nk
        D = aug_emb.shape[1]
        probe = seg.view(E, S, D)[:, :nk].unsqueeze(2)
        sup = torch.cat([probe, aug_emb.view(E, nk, ns_v, D)], 2).reshape(E * nk * (ns_v + 1), D)
        slots, nproto, off = [], [], [0]
        for p in plans:
            seen = {}
            for y in p['support_y']:
                sl_ = seen.setdefault(float(y), len(seen))
                slots += [sl_] * (ns_v + 1)
            nproto.append(len(seen))
            off.append(off[-1] + nk * (ns_v + 1))
        if self.classifier not in ('protonet', 'cosine'):  # SVM (host sklearn), KNN / unknown: raise as the reference
            sup_y = [np.repeat(np.asarray(p['support_y'], np.float32), ns_v + 1) for p in plans]
            return self._host_classify(torch.cat([sup, q_emb]), off, sup_y, [p['query_y'] for p in plans])
        pred, _ = _engine.match(q_emb, sup.contiguous(), t(off), t(slots), t(nproto), self.classifier)
        if debug is not None:  # concatenated over batches, in episode order
            for k, v in dict(seg=seg, pool=pool, sup=sup, q_emb=q_emb, pred=pred).items():
                debug[k] = torch.cat([debug[k], v]) if k in debug else v
        return pred.cpu().tolist()
