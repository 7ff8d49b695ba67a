"""Interleaved A/B of KMG_* settings for one device-resident spectrum / mismatch build in ONE
process on ONE output buffer (placement and clock drift cannot masquerade as a difference).
Usage: python3 tools/ab_env.py '{"kind": "sp", "n": 20000, "k": 8, "reps": 4, "steps": 10}'
                               '[{"KMG_SP_STORE": 1}, {"KMG_SP_STORE": 2}]'"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
from kmgram import _lib as L, encode as E, params as P  # noqa: E402


def main():
    cfg = json.loads(sys.argv[1])
    sets = json.loads(sys.argv[2])
    n, kind = cfg.get("n", 20000), cfg.get("kind", "sp")
    ctx = L.Context(0)
    codes, lens = E.synthetic(n, 101, seed=cfg.get("seed", 2))
    if kind == "sp":
        p, dt = P.make(L.KMG_SPECTRUM, k=cfg.get("k", 8)), L.KMG_I32
    elif kind == "ss":
        p, dt = P.make(L.KMG_SUBSTRING, k=cfg.get("k", 5), lbda=cfg.get("lbda", 0.5)), L.KMG_F64
    elif kind == "la":
        p, dt = P.make(L.KMG_LOCALALIGN, smith=cfg.get("smith", 0), la_mode=L.KMG_LA_INTENDED,
                       la_e=11, la_d=1, la_beta=0.5), L.KMG_F64
    elif kind == "wd":
        p, dt = P.make(L.KMG_WD, d=cfg.get("d", 5)), L.KMG_F64
    else:
        norm = cfg.get("norm", 1)
        p = P.make(L.KMG_MISMATCH, k=cfg.get("k", 9), m=1, window=101, normalize=norm)
        dt = L.KMG_F64 if norm else L.KMG_I32
    if cfg.get("f64"):
        dt = L.KMG_F64
    esz = 8 if dt == L.KMG_F64 else 4
    dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(dc, codes)
    ctx.h2d(dl, lens)
    do = ctx.dmalloc(n * n * esz)
    for rep in range(cfg.get("reps", 4)):
        for env in sets:
            for k in [k for k in os.environ if k.startswith("KMG_")]:
                del os.environ[k]
            os.environ.update({k: str(v) for k, v in env.items()})
            ctx.reload_tuning()
            ctx.gram_device(p, dc, dl, n, 101, 0, n, dt, do, n)
            ctx.synchronize()
            ctx.set_timing(2)
            ctx.timing_reset()
            steps = cfg.get("steps", 10)
            t = time.perf_counter()
            for _ in range(steps):
                ctx.gram_device(p, dc, dl, n, 101, 0, n, dt, do, n)
            ctx.synchronize()
            wall = (time.perf_counter() - t) / steps * 1e3
            tot, cnt = ctx.stage_stats("gram")
            mtot, mcnt = ctx.stage_stats("mirror")
            ctx.set_timing(0)
            print(json.dumps({"cfg": cfg, "env": env, "rep": rep, "ms": wall,
                              "gram_ms": tot / max(1, cnt),
                              "mirror_ms": mtot / mcnt if mcnt else 0.0}), flush=True)


if __name__ == "__main__":
    main()
