"""Child process of tests/test_gpu_rccl.py: the multi-GPU result exchange (distributed.py) over a real
RCCL communicator on the one GPU of the box (world size 1 -- RCCL refuses two ranks on one device).
Brings up the "nccl" process group exactly as bench.py does (device_id bound, 127.0.0.1 rendezvous),
broadcasts the weights, runs one search and gathers its results through both the blocking and the
overlapped all_gather, and prints one JSON line with what it checked.

    python tests/rccl_world1.py PORT
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(port):
    import numpy as np
    import torch
    import torch.distributed as dist

    from muzero_hanoi_amd import distributed as mdist
    from muzero_hanoi_amd import engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    init_s = time.perf_counter() - t0
    n, S, B = 4, 20, 4096
    torch.manual_seed(0)
    flat = engine.flat_weights(MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True).state_dict())
    got = mdist.broadcast_weights(flat, dev)
    assert np.array_equal(got, flat), "broadcast changed the weights"
    g = np.random.default_rng(5)
    st = g.integers(0, 3, (B, n))
    obs = np.zeros((B, 3 * n), np.float32)
    obs[np.arange(B)[:, None], np.arange(n) * 3 + st] = 1
    noise, tie, u = rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=7)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eng = engine.Engine(n, S, B, 33, device=0)
    eng.load_weights(got)
    out = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0,
                     deterministic=False, discount=0.8, eps=0.25)
    res = mdist.gather_results(out, B, 1)
    pend = mdist.gather_results_async(out, B, 1)
    pend[0].wait()
    res2 = mdist.unpack_results(pend[1])
    torch.cuda.synchronize(dev)
    checked = []
    for k in ("visits", "action", "root_q"):
        local = out[k].reshape(res[k].shape).to(res[k].dtype)
        assert torch.equal(res[k], local), k
        assert torch.equal(res2[k], local), k
        checked.append(k)
    assert int(res["visits"].sum(1).min()) == S
    backend = dist.get_backend()
    dist.destroy_process_group()
    eng.close()
    print(json.dumps({"backend": backend, "world_size": 1, "roots": B, "checked": checked,
                      "init_s": round(init_s, 3), "torch": torch.__version__}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]))
