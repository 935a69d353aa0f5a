#!/usr/bin/env python3
"""Headline benchmark: clips/s of the clip-embedding + one-shot matching path.

Workload (BASELINE.json configs[1], the metric's config): 5-way 1-shot episodes
sampled from the reference's test.list in the reference's RNG order, 8 segments x
seg_len 2 = 16 frames per clip at 224x224, ResNet-18 backbone, f32 arithmetic,
synthetic frames generated in HBM before the timed region.

One "step" = one batch of --episodes-per-step episodes per rank: every frame of
every clip through the backbone (one batched call), L2 + temporal mean per clip,
protonet matching of every episode.  Episodes are sharded e % world == rank; the
per-rank predictions are all-gathered once (RCCL) after the timed region.

Prints ONE JSON line (rank 0).  See DESIGN.md section "Measurement".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "embodied-one-shot-video-recognition_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402

MFMA_PEAK_TF = {"f32": 157.3, "bf16": 2516.6}  # MI355X dense peaks (MI355X_MICROARCH.md)
# f32x3 (EOSV_F32X3): every f32-accurate product is three bf16 MFMA products, so its ceiling in
# algorithmic (f32) FLOP/s is the bf16 dense peak / 3
MFMA_PEAK_TF["f32x3"] = round(MFMA_PEAK_TF["bf16"] / 3, 1)
ELEM_BYTES = {"f32": 4, "bf16": 2, "f32x3": 4}  # stored activation bytes per element (f32x3: the (hi, lo) pair)
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--episodes-per-step", type=int, default=100)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--n-way", type=int, default=5)
    ap.add_argument("--k-shot", type=int, default=1)
    ap.add_argument("--segments", type=int, default=8)
    ap.add_argument("--seg-len", type=int, default=2)
    ap.add_argument("--max-frames", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--list", default=None,
                    help="split list to sample episodes from (default: the reference's sources/data/test.list)")
    ap.add_argument("--cpu-baseline-sec", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train-leg", action="store_true",
                    help="skip the training-step leg (tools/bench_train.py's R50 finetune step; N = 1 and only "
                         "with the CPU baseline, so --no-cpu-baseline -- every profiling script's -- skips it too)")
    ap.add_argument("--layers", action="store_true", help="print per-layer conv timing to stderr")
    ap.add_argument("--config-label", default="BASELINE configs[1]",
                    help="which BASELINE.json config this run measures (tools/bench_configs.py sets it)")
    ap.add_argument("--parity-dump", default=None,
                    help="save the primary leg's timed-episode predictions and clip embeddings (npz) for "
                         "tools/offline_parity.py (the oracle over many more episodes than cpu_parity's sample)")
    ap.add_argument("--secondary-dtype", default="bf16,f32x3",
                    help="also time the same episodes with these backbone dtypes, comma-separated "
                         "('' or none to skip); the first is reported as 'secondary', the others as "
                         "'secondary_<dtype>'")
    return ap.parse_args()


def cpu_baseline(args, batch, T, emb, preds):
    """Oracle (fp32 torch-CPU restatement of the reference path) on a bounded sample of the last
    timed step's episodes; also checks the GPU leg against it on that sample (``cpu_parity``):
    predictions, clip embeddings, and the top-2 distance margin of every sampled episode."""
    sys.path.insert(0, REPO)
    from eosv import arch as arch_mod, synth  # noqa
    from oracle import harness_ref, resnet_ref  # noqa  (checker / CPU baseline only)
    from scipy.spatial.distance import cdist

    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    model = resnet_ref.build_model(args.arch, synth.synth_state_dict(arch_mod.SPECS[args.arch], 64, 0))

    def load(vi, support):
        ids, n_all = synth.clip_frame_ids(vi, T)
        v = torch.from_numpy(synth.synth_video(vi.split("/")[0], vi, ids, args.res, args.res))
        return v, v.shape[0]

    t_load = 0.0
    clips = frames = done = 0
    pred_equal, emb_rel, margins = 0, 0.0, []
    t0 = time.perf_counter()
    for j, ep in enumerate(batch.episodes):
        tl = time.perf_counter()
        vids = [load(v, True) for v in ep["support"]] + [load(ep["query"], False)]
        t_load += time.perf_counter() - tl
        sx = [v for v, _ in vids[:-1]]
        sf = [n for _, n in vids[:-1]]
        s_emb = harness_ref.epoch_features(model, sx, True, sf)
        q_emb = harness_ref.epoch_features(model, [vids[-1][0]], True)
        clips += len(vids)
        frames += sum(n for _, n in vids)
        done += 1
        tc = time.perf_counter()
        # checker (excluded from the CPU time like the frame generation)
        sy = np.array(ep["support_y"], np.float32)
        ref_pred = harness_ref.protonet_predict(s_emb, sy, q_emb, np.array([ep["query_y"]], np.float32))[0][0]
        pred_equal += int(ref_pred == int(preds[j]))
        s0, s1 = int(batch.sup_off[j]), int(batch.sup_off[j + 1])
        got = np.concatenate([emb[s0:s1], emb[batch.n_support + j][None]])
        ref = np.concatenate([s_emb, q_emb])
        emb_rel = max(emb_rel, float((np.abs(got - ref).max(1) / np.abs(ref).max(1)).max()))
        _, protos = harness_ref.prototypes(s_emb, sy)
        d = np.sort(cdist(q_emb.astype(np.float64), protos.astype(np.float64))[0])
        margins.append((d[1] - d[0]) / d[0])
        t_load += time.perf_counter() - tc
        if j % 4 == 3:  # progress on stderr: a long CPU sample must not look hung to a watchdog
            print(f"cpu_baseline: {j + 1} episodes, {time.perf_counter() - t0 - t_load:.0f}s", file=sys.stderr, flush=True)
        if time.perf_counter() - t0 - t_load > args.cpu_baseline_sec:
            break
    el = time.perf_counter() - t0 - t_load
    base = {"value": round(clips / el, 3), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"{done} episodes ({clips} clips, {frames} frames) of the last timed step through "
                      f"oracle/ (torch-CPU fp32 restatement of network_test.py:49-68 + classifier.py), "
                      f"synthetic-frame generation and the parity check excluded; {el:.1f}s"}
    parity = {"episodes": done, "pred_equal": pred_equal, "max_emb_rel": float(f"{emb_rel:.3g}"),
              "min_top2_margin": float(f"{min(margins):.3g}"),
              "near_ties": int(sum(m < 1e-5 for m in margins)),
              "against": f"{args.dtype} leg, last timed step"}
    return base, parity


def run_timed(args, engine, arch_mod, synth, batches, dtype, local, dist, keep_emb=False):
    """Warmup + timed region for one backbone dtype; returns (max-over-ranks elapsed_s, every rank's
    elapsed_s, preds, per-layer profile, clip embeddings of the last step; with keep_emb those of
    every timed step, concatenated)."""
    bb = engine.Backbone(args.arch, dtype, args.res, args.res, max_frames=args.max_frames, device=local)
    bb.load_state_dict(synth.synth_state_dict(arch_mod.SPECS[args.arch], 64, 0))
    feat = torch.empty(max(d.batch.n_frames for d in batches), bb.D, device=f"cuda:{local}")
    for s in range(args.warmup):
        d = batches[s]
        engine.run_episodes(bb, d, "protonet", True, feat=feat[:d.batch.n_frames])
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    bb.profile(True)
    preds, embs = [], []
    t0 = time.perf_counter()
    for s in range(args.warmup, len(batches)):
        d = batches[s]
        p, emb, _ = engine.run_episodes(bb, d, "protonet", True, feat=feat[:d.batch.n_frames])
        preds.append(p)
        if keep_emb:
            embs.append(emb.clone())  # the next step reuses the output buffer
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = bb.profile_read()
    bb.profile(False)
    bb.close()
    from eosv import dist as edist
    per_rank = edist.gather_values(elapsed)
    if keep_emb:
        return max(per_rank), per_rank, torch.cat(preds), prof, torch.cat(embs).cpu().numpy()
    return max(per_rank), per_rank, torch.cat(preds), prof, emb.cpu().numpy()


def traffic_key(args):
    """The workload a PMC traffic profile belongs to: arch, frame size and BASELINE config."""
    return f"{args.arch}@{args.res}x{args.res}/{args.config_label}"


def measured_traffic(dtype, key):
    """HBM bytes per conv launch from a profiles/<tag>_traffic.json written by tools/traffic_json.py
    from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this command at this dtype
    (tools/gpu_traffic.sh; the figure covers exactly the timed region's conv-family launches of the
    profiled run, the same launches its traffic_algorithmic covers).  EOSV_TRAFFIC_PROFILE names a
    specific file, else the newest matching one.  None unless the workload key, the dtype, the
    kernel sources (src_sha16 = eosv._lib.source_digest()) and the build configuration (lib_kind:
    the release library, not the profiling or a variant build) all match: counters measured on
    other kernels are never attached.  (The library's own bytes, lib_sha16, are recorded by
    tools/traffic_json.py for information only: r05 hashed them into src_sha16, so a rebuild of the
    same sources detached every profile.)"""
    import glob
    from eosv._lib import library_kind, source_digest
    paths = [os.environ["EOSV_TRAFFIC_PROFILE"]] if os.environ.get("EOSV_TRAFFIC_PROFILE") else \
        sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), reverse=True)
    digest, kind = source_digest(), library_kind()
    for path in paths:
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        if d.get("key") == key and d.get("src_sha16") == digest and d.get("lib_kind", "release") == kind and dtype in d:
            return d[dtype], os.path.relpath(path, REPO)
    return None, None


def algorithmic_bytes_per_launch(args, arch_mod, dtype, frames, prof):
    """Conv-family algorithmic bytes per launch over the timed region's launches: every launch's
    input + output (+ residual or folded-downsample input) map once per frame and its weights once
    per launch (arch.conv_launch_bytes: the fused stem + pool reads the f32 frame and writes the
    pooled map); a bf16 conv1 fused into the previous conv3 launch (pair kernels) adds its bytes
    less its never-read input map (as layer_bounds)."""
    ms, fl, nl = prof
    spec = arch_mod.SPECS[args.arch]
    layers = arch_mod.fuse_bneck_bytes(arch_mod.conv_launch_bytes(spec, args.res, args.res, ELEM_BYTES[dtype]), spec, nl)
    total = 0.0
    for i in range(min(len(layers), len(nl))):
        pf, wb, pin = layers[i]
        if nl[i]:
            total += frames * pf + int(nl[i]) * wb
        elif pf:  # fused into the previous launch: same frames, its input map never read
            j = max((k for k in range(i) if nl[k]), default=None)
            if j is not None:
                total += frames * (pf - pin) + int(nl[j]) * wb
    return total / max(1, int(nl.sum()))


def layer_bounds(prof, dtype, args, arch_mod, frames):
    """Per-launch roofline of the timed region: for every conv layer, its floor time is
    max(algorithmic FLOPs / MFMA peak, algorithmic bytes (arch.conv_launch_bytes) / HBM peak);
    frac = sum of floors / sum of measured HIP-event times.  A layer is 'hbm'-bound when the byte
    floor is the larger (R50's 1x1 convs at K = 64..256, the bf16 stage-1 maps)."""
    ms, fl, nl = prof
    spec = arch_mod.SPECS[args.arch]
    layers = arch_mod.fuse_bneck_bytes(arch_mod.conv_launch_bytes(spec, args.res, args.res, ELEM_BYTES[dtype]), spec, nl)
    peak = MFMA_PEAK_TF[dtype] * 1e12
    nlay = min(len(ms), len(layers))
    # a conv with no launch of its own but bytes (bf16 bottleneck conv1 fused into the previous
    # block's conv3 launch, pair1x1_bf16.hip; its FLOPs are in that record): its bytes less its
    # input map (never re-read) join the launch it was fused into
    eb = [[float(layers[i][0]), float(layers[i][1])] for i in range(nlay)]
    for i in range(nlay):
        if not nl[i] and layers[i][0]:
            j = max((k for k in range(i) if nl[k]), default=None)
            if j is not None:
                eb[j][0] += layers[i][0] - layers[i][2]
                eb[j][1] += layers[i][1]
    t_meas = t_floor = t_hbm_layers = 0.0
    n_hbm = n = 0
    worst = None
    for i in range(nlay):
        if not nl[i]:
            continue
        pf, wb = eb[i]
        t_m = float(fl[i]) / peak * 1e3
        t_b = (frames * pf + int(nl[i]) * wb) / (HBM_PEAK_GBPS * 1e9) * 1e3
        fl_i = max(t_m, t_b)
        t_meas += float(ms[i])
        t_floor += fl_i
        n += 1
        if t_b > t_m:
            n_hbm += 1
            t_hbm_layers += float(ms[i])
        if worst is None or fl_i / float(ms[i]) < worst[1]:
            worst = (i, fl_i / float(ms[i]), "hbm" if t_b > t_m else "mfma")
    if not n:
        return None
    return {"frac": round(t_floor / t_meas, 4), "layers": n, "hbm_bound_layers": n_hbm,
            "hbm_bound_time_share": round(t_hbm_layers / t_meas, 4),
            "worst_layer": {"id": worst[0], "frac": round(worst[1], 4), "bound": worst[2]},
            "hbm_peak": HBM_PEAK_GBPS, "mfma_peak": MFMA_PEAK_TF[dtype],
            "definition": "sum over conv layers of max(FLOPs / MFMA peak, algorithmic bytes / HBM peak) "
                          "/ sum of measured per-layer HIP-event times (layer ids: arch.conv_launch_bytes order)"}


def print_layers(prof, tag):
    ms, fl, nl = prof
    for i in range(len(ms)):
        if nl[i]:
            print(f"[{tag}] layer {i:3d}: {ms[i] / nl[i]:8.3f} ms/launch  {fl[i] / ms[i] / 1e9:7.2f} TF/s",
                  file=sys.stderr)


def roofline(prof, dtype, args=None, arch_mod=None, frames=None):
    ms, fl, nl = prof
    conv_ms, conv_fl = float(ms.sum()), float(fl.sum())
    achieved = conv_fl / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    peak = MFMA_PEAK_TF[dtype]
    out = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
           "frac": round(achieved / peak, 4), "traffic": None,
           "kernel": f"conv_{dtype}_kernel family: all {int(nl.sum())} conv launches of the timed region, "
                     f"summed algorithmic FLOPs / summed HIP-event durations on the launch stream"}
    if dtype == "f32x3":
        out["kernel"] += ("; f32x3 = conv_bf16 kernels on the split (hi, lo) layout + the split-bf16 fused "
                          "stem (stem_pool_x3_cb_kernel), algorithmic (f32) FLOPs; peak = bf16 dense peak / 3")
    if args is not None and nl.sum() > 0:
        out["conv_launches"] = int(nl.sum())
        out["traffic_key"] = traffic_key(args)
        tr, src = measured_traffic(dtype, out["traffic_key"])
        out["traffic"] = tr["hbm_bytes_per_launch"] if tr else None
        out["traffic_unit"] = "HBM bytes per conv launch"
        out["traffic_algorithmic"] = round(algorithmic_bytes_per_launch(args, arch_mod, dtype, frames, prof))
        out["traffic_source"] = src
        if tr:  # the profiled run's own figures, over the same launches as its measured bytes
            out["traffic_profiled_run"] = {k: tr[k] for k in ("launches", "hbm_bytes_per_launch",
                                                               "algorithmic_bytes_per_launch", "ratio") if k in tr}
        out["per_layer_bound"] = layer_bounds(prof, dtype, args, arch_mod, frames)
    return out


def spawn_ranks(n):
    """``--gpus N`` without a launcher: start N rank processes (RANK / LOCAL_RANK / WORLD_SIZE,
    rendezvous on 127.0.0.1) and wait for them.  This process never touches the GPU (no HIP
    call happens before here), and the ranks are children, not an exec of this process.
    Rank 0 prints the JSON line; the exit code is the first failing rank's."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc), 0)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} ranks", file=sys.stderr)
    # one rank per GPU; more ranks than devices share them round-robin (gloo rehearsals only)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    # a process group for N > 1, or at N = 1 when a backend is named (EOSV_DIST_BACKEND=nccl runs
    # the RCCL path -- barrier, all-gathers, all-reduce -- on one GPU; MASTER_ADDR / MASTER_PORT
    # must then be set, as under a launcher)
    dist = world > 1 or bool(os.environ.get("EOSV_DIST_BACKEND"))
    torch.cuda.set_device(local)
    if dist:
        import torch.distributed as tdist
        backend = os.environ.get("EOSV_DIST_BACKEND") or "nccl"  # nccl == RCCL on ROCm
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:  # N = 1 without a launcher: a free local port
            if world > 1:  # every rank would pick its own port and the rendezvous would hang
                sys.exit("bench.py: WORLD_SIZE > 1 needs MASTER_PORT (torch.distributed.run or "
                         "`bench.py --gpus N` set it)")
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        tdist.init_process_group(backend, rank=rank, world_size=world,
                                 device_id=torch.device("cuda", local) if backend == "nccl" else None)
    from eosv import arch as arch_mod, dist as edist, engine, episodes as ep_mod, synth  # noqa

    T = args.segments * args.seg_len
    E = args.episodes_per_step
    n_steps = args.warmup + args.steps
    lines = open(args.list).readlines() if args.list else None
    plans = ep_mod.plan_episodes(E * n_steps * world, args.n_way, args.k_shot, "test", seed=args.seed, lines=lines)
    mine_idx = edist.shard_indices(len(plans), rank, world)  # episode e runs on rank e % world
    batches = []
    for s in range(n_steps):
        b = engine.build_episode_batch([plans[e] for e in mine_idx[s * E:(s + 1) * E]], T)
        batches.append(engine.DeviceEpisodes(b, args.res, args.res, device=local))
    torch.cuda.synchronize()
    timed_idx = mine_idx[args.warmup * E:]

    dump = bool(args.parity_dump) and world == 1
    elapsed, per_rank_elapsed, pred, prof, emb = run_timed(args, engine, arch_mod, synth, batches, args.dtype, local, dist,
                                                           keep_emb=dump)
    if dump:  # every timed step's embeddings: the last step's are the tail (cpu_baseline's sample)
        all_emb = emb
        emb = all_emb[-batches[-1].batch.n_clips:]
        np.savez_compressed(args.parity_dump, pred=pred.cpu().numpy().astype(np.int64), emb=all_emb,
                            timed_idx=np.asarray(timed_idx, np.int64), n_plans=len(plans),
                            args=json.dumps({k: v for k, v in vars(args).items()}))
    per_rank_clips = [int(v) for v in edist.gather_values(sum(d.batch.n_clips for d in batches[args.warmup:]))]
    clips = sum(per_rank_clips)
    frames_rank = sum(d.batch.n_frames for d in batches[args.warmup:])
    frames = edist.sum_over_ranks(frames_rank)
    # (episode, prediction) pairs: ONE all-gather over xGMI (RCCL) after the timed region
    preds = edist.gather_predictions(timed_idx, pred.cpu().numpy(), len(plans))
    timed = preds >= 0
    qy = np.array([p["query_y"] for p in plans])
    acc = float((preds[timed] == qy[timed]).mean())

    legs = []
    for dt2 in [d for d in (args.secondary_dtype or "").split(",") if d and d not in ("none", args.dtype)]:
        el2, _, pred2, prof2, emb2 = run_timed(args, engine, arch_mod, synth, batches, dt2, local, dist)
        # clip embeddings of the last step vs the f32 primary: max over clips of
        # max|e - e_f32| / max|e_f32| (the north star's 1e-4 relative bound, tests/test_gpu_parity.py)
        if args.layers and rank == 0:
            print_layers(prof2, dt2)
        emb_rel = float((np.abs(emb2 - emb).max(1) / np.maximum(np.abs(emb).max(1), 1e-30)).max())
        preds2 = edist.gather_predictions(timed_idx, pred2.cpu().numpy(), len(plans))
        legs.append({"dtype": dt2, "value": round(clips / el2, 2), "unit": "clips/s",
                     "ms_per_step": round(el2 / args.steps * 1e3, 3),
                     "prediction_agreement_vs_primary": round(float((preds2[timed] == preds[timed]).mean()), 4),
                     "episode_acc": round(float((preds2[timed] == qy[timed]).mean()), 4),
                     "embedding_max_rel_vs_primary": float(f"{emb_rel:.3g}"),
                     "roofline": roofline(prof2, dt2, args, arch_mod, frames_rank)})

    if rank == 0:
        ms, fl, nl = prof
        gflop_frame = 2 * arch_mod.conv_macs_per_frame(arch_mod.SPECS[args.arch], args.res, args.res) / 1e9
        rl = roofline(prof, args.dtype, args, arch_mod, frames_rank)
        rl["end_to_end_tflops"] = round(frames * gflop_frame / elapsed / 1e3, 2)
        rl["flop_per_frame"] = round(gflop_frame * 1e9)
        out = {
            # BASELINE.json's metric string at the default config; the config-4/5 shapes name theirs
            "metric": f"clips/sec/GPU ({args.res}\u00b2, {args.segments}-seg) + {args.n_way}-way-{args.k_shot}-shot "
                      "episode acc vs reference",
            "value": round(clips / elapsed, 2),  # whole job: all ranks' clips / max-over-ranks time
            "unit": "clips/s",
            "value_per_gpu": round(clips / elapsed / world, 2),
            # the metric string is BASELINE.json's; 'value' is the driver contract's whole-job figure
            "value_semantics": "value = all ranks' clips / max-over-ranks time (whole job over n_gpus); "
                               "the metric's per-GPU figure is value_per_gpu = value / n_gpus",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic frames (deterministic, generated in HBM) + random-init weights of the "
                    "reference architecture; episodes from "
                    + (os.path.relpath(args.list, REPO) if args.list else "the reference's test.list")
                    + " in the reference's RNG order",
            "config": {"workload": f"test_network_baseline {args.n_way}-way {args.k_shot}-shot, "
                                   f"{args.segments} seg x {args.seg_len} frames, {args.arch}, "
                                   f"{args.res}x{args.res}, {args.dtype} ({args.config_label})",
                       "episodes_per_step_per_gpu": E, "episodes_timed": E * args.steps * world,
                       "frames_per_clip": T, "parallelism": f"episode-sharded dp{world}"},
            "frames_per_s": round(frames / elapsed, 1),
            # self-verifying multi-rank record: what the process group reports, and every rank's share
            "dist": dict(edist.describe(), launched_world_size=world,
                         per_rank_clips=per_rank_clips,
                         per_rank_elapsed_s=[round(v, 6) for v in per_rank_elapsed],
                         collective="all_gather of (episode, prediction) int64 pairs after the timed region"),
            "episode_acc": round(acc, 4),
            "roofline": rl,
            "cpu_baseline": None,
        }
        for i, leg in enumerate(legs):
            out["secondary" if i == 0 else "secondary_" + leg["dtype"]] = leg
        if args.layers:
            print_layers(prof, args.dtype)
        if not args.no_train_leg and not args.no_cpu_baseline and world == 1:
            # the reference's other entry point (network_train.py finetune step), after
            # the timed region: R50, its batch of 6 clips x 16 frames at 224x224, f32, 1 + 5 steps
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from bench_train import measure
            out["training"] = measure(device=local)[0]
        if not args.no_cpu_baseline and world == 1:
            last = batches[-1].batch
            out["cpu_baseline"], out["cpu_parity"] = cpu_baseline(args, last, T, emb, pred[-len(last.episodes):].cpu().numpy())
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
