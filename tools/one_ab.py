"""Same-box A/B of library builds on the latency kernel (mzh_search_one_kernel): HIP-event time of one search
launch, median of 60 after warm-up, for the run_mcts shape (N=3, S=25, 1 root) and N=4, S=50 at 1 and 256 roots;
libraries alternated ABBA over the rounds, each measured in its own process.

    python tools/one_ab.py muzero-hanoi_amd/libmzh.so muzero-hanoi_amd/libmzh_base.so [--rounds 2] [--out F]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = ((3, 25, 1), (4, 50, 1), (4, 50, 256))


def child():
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    import bench
    from muzero_hanoi_amd import engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    out = {}
    for n, S, B in SHAPES:
        torch.manual_seed(0)
        net = MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)
        eng = engine.Engine(n, S, B, 33)
        eng.load_weights(engine.flat_weights(net.state_dict()))
        obs = torch.from_numpy(bench.random_roots(n, B, 0)).cuda()
        noise, tie, u = (torch.from_numpy(x).cuda() for x in rng.synthetic_draws(B, deterministic=False, alpha=0.25,
                                                                                   seed=0))
        res = eng.alloc_search_outputs(B, S)
        fn = lambda: eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, out=res,
                                kernel="one")
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(60)]
        for s, e in ev:
            s.record()
            fn()
            e.record()
        torch.cuda.synchronize()
        out[f"n{n}s{S}b{B}"] = float(np.median([s.elapsed_time(e) for s, e in ev]))
        eng.close()
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.child:
        return child()
    rows = []
    for r in range(a.rounds):
        order = a.libs if r % 2 == 0 else a.libs[::-1]
        for lib in order:
            env = dict(os.environ, MZH_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                raise SystemExit(p.returncode)
            row = dict(json.loads(p.stdout.strip().splitlines()[-1]), lib=os.path.basename(lib), round=r)
            rows.append(row)
            print(json.dumps(row), flush=True)
    summary = {}
    for lib in a.libs:
        b = os.path.basename(lib)
        summary[b] = {k: sorted(x[k] for x in rows if x["lib"] == b) for k in rows[0] if k.startswith("n")}
    print(json.dumps(summary))
    if a.out:
        json.dump({"rows": rows, "summary_ms": summary}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
