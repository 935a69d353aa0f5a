#!/usr/bin/env python3
"""Oracle parity of a bench run over many more episodes than its cpu_parity sample.

The box's CPU share (16 threads) runs the oracle on a bounded sample inside bench.py (cpu_baseline,
~10-30 s); for the config lines whose episodes are large (C5: 1,664 frames of R101 at 256x256 per
episode, ~1 min each on 16 cores) that sample is one or two episodes.  This tool takes the GPU
leg's predictions and clip embeddings saved by ``bench.py --parity-dump`` (every timed episode)
and re-runs the oracle on the first N timed episodes on THIS machine's CPU, untimed: the same
plans (the plan service, same seed / list / shape), the same synthetic frames (eosv/synth.py, the
generator the device path restates bit for bit) and the same synthetic weights.

  python tools/offline_parity.py profiles/r05_c5_dump.npz 20 [out.json]

Prints / writes {"episodes", "pred_equal", "max_emb_rel", "min_top2_margin", "near_ties", ...}.
The oracle (oracle/, CPU restatement of network_test.py:49-68 + classifier.py) is the checker
only; nothing here is timed or reported as a throughput.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else None
    from scipy.spatial.distance import cdist

    from eosv import arch as arch_mod, engine, episodes as ep_mod, synth
    from oracle import harness_ref, resnet_ref

    d = np.load(path, allow_pickle=False)
    args = json.loads(str(d["args"]))
    pred, emb, timed_idx = d["pred"], d["emb"], d["timed_idx"]
    T = args["segments"] * args["seg_len"]
    E = args["episodes_per_step"]
    lines = None
    if args.get("list"):
        lp = args["list"]
        if not os.path.exists(lp):  # a path on the GPU box (its scratch copy of the repo)
            lp = os.path.join(REPO, lp[lp.rindex("tests/golden/"):]) if "tests/golden/" in lp else lp
        lines = open(lp).readlines()
    plans = ep_mod.plan_episodes(int(d["n_plans"]), args["n_way"], args["k_shot"], "test", seed=args["seed"],
                                 lines=lines)
    # the timed steps' batches, in the order bench.py ran them (world 1: episodes in plan order)
    steps = [timed_idx[i:i + E] for i in range(0, len(timed_idx), E)]
    batches = [engine.build_episode_batch([plans[e] for e in st], T) for st in steps]
    torch.set_num_threads(len(os.sched_getaffinity(0)))
    model = resnet_ref.build_model(args["arch"], synth.synth_state_dict(arch_mod.SPECS[args["arch"]], 64, 0))

    def load(vi):
        ids, _ = synth.clip_frame_ids(vi, T)
        v = torch.from_numpy(synth.synth_video(vi.split("/")[0], vi, ids, args["res"], args["res"]))
        return v, v.shape[0]

    done = pred_equal = 0
    emb_rel, margins = 0.0, []
    row0 = 0
    t0 = time.time()
    for bi, b in enumerate(batches):
        for j, ep in enumerate(b.episodes):
            if done >= n:
                break
            vids = [load(v) for v in ep["support"]] + [load(ep["query"])]
            s_emb = harness_ref.epoch_features(model, [v for v, _ in vids[:-1]], True, [c for _, c in vids[:-1]])
            q_emb = harness_ref.epoch_features(model, [vids[-1][0]], True)
            sy = np.array(ep["support_y"], np.float32)
            ref = harness_ref.protonet_predict(s_emb, sy, q_emb, np.array([ep["query_y"]], np.float32))[0][0]
            gi = bi * E + j
            pred_equal += int(int(ref) == int(pred[gi]))
            s0, s1 = int(b.sup_off[j]), int(b.sup_off[j + 1])
            got = np.concatenate([emb[row0 + s0:row0 + s1], emb[row0 + b.n_support + j][None]])
            want = np.concatenate([s_emb, q_emb])
            emb_rel = max(emb_rel, float((np.abs(got - want).max(1) / np.abs(want).max(1)).max()))
            _, protos = harness_ref.prototypes(s_emb, sy)
            dd = np.sort(cdist(q_emb.astype(np.float64), protos.astype(np.float64))[0])
            margins.append(float((dd[1] - dd[0]) / dd[0]))
            done += 1
            print(f"episode {done}: ref {int(ref)} gpu {int(pred[gi])} emb_rel {emb_rel:.3g} "
                  f"({time.time() - t0:.0f}s)", flush=True)
        row0 += b.n_support + len(b.episodes)
        if done >= n:
            break
    res = {"episodes": done, "pred_equal": pred_equal, "max_emb_rel": float(f"{emb_rel:.3g}"),
           "min_top2_margin": float(f"{min(margins):.3g}"), "near_ties": int(sum(m < 1e-5 for m in margins)),
           "against": f"{args['dtype']} leg of {os.path.basename(path)} (bench.py --parity-dump), first {done} "
                      f"timed episodes, oracle on this machine's CPU (untimed)",
           "workload": {k: args[k] for k in ("arch", "res", "n_way", "k_shot", "segments", "seg_len", "seed",
                                             "dtype", "config_label")}}
    print(json.dumps(res))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
