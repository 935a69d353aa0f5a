"""The r05 training passes against the r04 ones they replace (EOSV_TRAIN_R04=1), same inputs, every
output bitwise equal:
  * batch-norm statistics with 4 rows per lane loaded ahead (same row chunks), the backward's ReLU
    mask from the forward's mask bytes (no y), dx from the residual gradient when it is written:
    y, saved mean and inverse std, running estimates, dx, dgamma, dbeta, residual gradient;
  * im2col with four elements and one 16-byte store per lane, col2im over four channels per lane.
Needs the profiling build (EOSV_LIBRARY=libeosv_prof.so), which reads the switch per call.
usage: python tools/train_r05_check.py  -> prints 'train_r05_check: <n> cases, <k> differing'"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))

from eosv._lib import check, lib, stream_ptr  # noqa: E402

# (P rows, C channels, relu, residual, dres): R50 layer shapes at 6 clips x 16 frames / 4 (layer1
# conv1 / conv3, layer4), ragged row counts (tails of the 4-row groups), the scalar V = 1 path (C = 6)
CASES = [(75265, 64, True, False, False), (75263, 256, True, True, True), (1177, 2048, True, True, True),
         (4704, 512, False, False, False), (10007, 6, True, True, True), (10007, 6, True, False, False),
         (97, 40, True, False, True)]


def run(L, P, C, relu, res, dres, seed, mask=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(P, C, device="cuda", generator=g) * 2 + 0.5
    r = torch.randn(P, C, device="cuda", generator=g)
    dy = torch.randn(P, C, device="cuda", generator=g)
    gam = torch.rand(C, device="cuda", generator=g) + 0.5
    bet = torch.randn(C, device="cuda", generator=g)
    rm, rv = torch.randn(C, device="cuda", generator=g), torch.rand(C, device="cuda", generator=g) + 0.5
    y, mean, inv = torch.empty_like(x), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    mk = torch.empty(P * C, dtype=torch.uint8, device="cuda") if mask else None
    work = torch.empty(int(L.eosv_bn_workspace_bytes(C)) // 4 + 4, device="cuda")
    s = stream_ptr()
    check(L.eosv_bn_train_forward(x.data_ptr(), P, C, gam.data_ptr(), bet.data_ptr(), 1e-5, 0.1, rm.data_ptr(),
                                  rv.data_ptr(), r.data_ptr() if res else 0, int(relu), y.data_ptr(),
                                  mk.data_ptr() if mask else None,
                                  mean.data_ptr(), inv.data_ptr(), work.data_ptr(), s), "eosv_bn_train_forward")
    dx, dg, db = torch.empty_like(x), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    dr = torch.empty_like(x) if dres else None
    ymk = (None, mk.data_ptr()) if mask and relu else (y.data_ptr(), None)
    check(L.eosv_bn_train_backward(dy.data_ptr(), *ymk, int(relu), x.data_ptr(), P, C, gam.data_ptr(),
                                   mean.data_ptr(), inv.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                   dr.data_ptr() if dres else 0, work.data_ptr(), s), "eosv_bn_train_backward")
    torch.cuda.synchronize()
    outs = [y, mean, inv, rm, rv, dx, dg, db] + ([dr] if dres else [])
    return [t.cpu() for t in outs]


# (N, H, W, C, k, stride, pad): the R50 stem, odd totals (tails of the 4-element groups), the
# strided 3x3 / 1x1 dgrads of layer2-4, and C % 4 != 0 (col2im's scalar kernel)
COL_CASES = [(4, 224, 224, 3, 7, 2, 3), (3, 9, 11, 3, 3, 2, 1), (2, 56, 56, 128, 3, 2, 1), (2, 28, 28, 256, 1, 2, 0),
             (2, 14, 14, 1024, 1, 2, 0), (1, 13, 9, 6, 3, 2, 1), (1, 7, 7, 5, 3, 1, 1)]


def run_col(L, N, H, W, C, k, stride, pad, seed):
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N * H * W * C, device="cuda", generator=g)
    dcol = torch.randn(N * Ho * Wo * k * k * C, device="cuda", generator=g)
    col, dx = torch.full_like(dcol, float("nan")), torch.full_like(x, float("nan"))
    s = stream_ptr()
    check(L.eosv_im2col(x.data_ptr(), N, H, W, C, k, k, stride, pad, col.data_ptr(), s), "eosv_im2col")
    check(L.eosv_col2im(dcol.data_ptr(), N, H, W, C, k, k, stride, pad, dx.data_ptr(), s), "eosv_col2im")
    torch.cuda.synchronize()
    return [col.cpu(), dx.cpu()]


def main():
    L = lib()
    bad = 0
    for i, (P, C, relu, res, dres) in enumerate(CASES):
        got = {}
        for old in ("1", "0"):
            os.environ["EOSV_TRAIN_R04"] = old
            # r05 side: the forward's ReLU mask bytes feed the backward (no y)
            got[old] = run(L, P, C, relu, res, dres, 11 + i, mask=old == "0")
        names = ["y", "mean", "invstd", "running_mean", "running_var", "dx", "dgamma", "dbeta", "dres"]
        diff = [n for n, a, b in zip(names, got["1"], got["0"]) if not torch.equal(a, b)]
        bad += bool(diff)
        print(f"bn P {P} C {C} relu {relu} res {res} dres {dres}: {'differ ' + ','.join(diff) if diff else 'equal'}")
    for i, case in enumerate(COL_CASES):
        got = {}
        for old in ("1", "0"):
            os.environ["EOSV_TRAIN_R04"] = old
            got[old] = run_col(L, *case, 31 + i)
        # equal_nan: a NaN left in the output would mean an unwritten element on both sides
        diff = [n for n, a, b in zip(["col", "dx"], got["1"], got["0"])
                if not torch.equal(a, b) or bool(torch.isnan(b).any())]
        bad += bool(diff)
        print(f"im2col/col2im {case}: {'differ ' + ','.join(diff) if diff else 'equal'}")
    os.environ.pop("EOSV_TRAIN_R04", None)
    print(f"train_r05_check: {len(CASES) + len(COL_CASES)} cases, {bad} differing")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
