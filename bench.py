"""Benchmark: MCTS simulations/sec of the fused batched search (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]                       # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W             # N>1, one rank per GPU

Workload: 4-disk Hanoi, 50 simulations per move, 65,536 random non-goal root states per GPU -- the
metric's 65k-root batch on every GPU (weak scaling: N GPUs search N independent 65k-root batches;
BASELINE configs[2], the same batch sharded 8 ways, is `--roots-per-gpu 8192`), MuZeroNet(TD_return=True) with
random-init weights (torch.manual_seed(0), broadcast once), training-like search parameters
(gamma 0.8, Dirichlet alpha 0.25 / eps 0.25, T=1, stochastic).  One step = one mzh_search launch
over every root on the rank (root inference + 50 x {select, MFMA MLP, backup} + play policy),
followed by the RCCL all_gather of the visit histograms (north_star's only exchange).  Inputs are
resident in HBM before timing starts.

Rank 0 prints ONE JSON line (contract in the task statement) including `roofline` for the
fused search kernel (fp32-MFMA bound; achieved = algorithmic matmul FLOPs per launch / mean
launch time from HIP events on the launch stream) and `cpu_baseline` (the reference algorithm's
Python restatement, oracle/py_port.py, on one host core over a bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (matrix), spec
MLP_FLOP_PER_SIM = 203_776     # recurrent_inference matmul FLOPs (2 x 101,888 MAC)


def root_flops(n_disks):
    return 2 * (768 * n_disks + 59_136)  # initial_inference matmul FLOPs


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--roots-per-gpu", type=int, default=65536)
    p.add_argument("--sims", type=int, default=50)
    p.add_argument("--disks", type=int, default=4)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-gather", action="store_true")
    p.add_argument("--kernel", choices=["auto", "coop", "wave", "wave16"], default="auto")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, one rank per GPU); gloo lets ranks share a GPU to rehearse the N>1 path")
    p.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    return p.parse_args()


def random_roots(n_disks, B, seed):
    """uniform over the 3^N states excluding the goal (env/hanoi.py:103-109 distribution)"""
    g = np.random.default_rng(seed)
    goal = 3 ** n_disks - 1
    idx = g.integers(0, goal, size=B)  # [0, goal) == every state but the goal (index 3^N - 1)
    st = np.stack([(idx // 3 ** (n_disks - 1 - d)) % 3 for d in range(n_disks)], 1)
    obs = np.zeros((B, 3 * n_disks), np.float32)
    obs[np.arange(B)[:, None], np.arange(n_disks) * 3 + st] = 1.0
    return obs


def cpu_baseline(n_disks, S, seconds, seed):
    """oracle/py_port.py (object tree, batch-1 torch-CPU MLP, NumPy RNG) on one core."""
    from muzero_hanoi_amd.networks import MuZeroNet
    from oracle import py_port

    torch.set_num_threads(1)
    torch.manual_seed(seed)
    net = MuZeroNet(3 * n_disks, 6, 0.002, "cpu", TD_return=True)
    pnet = py_port.PortNet({k: v.numpy() for k, v in net.state_dict().items()})
    obs = random_roots(n_disks, 4096, seed + 99).astype(np.float64)
    np.random.seed(seed)
    roots = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and roots < len(obs):
        m = py_port.PortMCTS(0.8, 0.25, S)
        m.run_mcts(obs[roots], pnet, 1.0, False)
        roots += 1
    dt = time.perf_counter() - t0
    return {"value": roots * S / dt, "unit": "sims/s", "cores": 1, "kind": "port",
            "sample": f"{roots} roots x {S} sims, {n_disks}-disk, fresh MCTS per root, T=1 stochastic, "
                      f"{dt:.1f} s on 1 host core (torch threads=1); oracle/py_port.py restates "
                      f"MCTS/mcts.py + networks.py and matches the reference's visits bit-exactly"}


def cpu_baseline_selfplay(n_disks, S, max_steps, seconds, net_state, start_state):
    """Self-play CPU baseline (tools/bench_selfplay.py): the reference algorithm on one host core --
    oracle/py_port.py's object-tree MCTS (batch-1 torch-CPU MLP, NumPy RNG) and the C env
    restatement -- playing episodes from start_state(k) until done or `seconds` run out.
    Returns (decisions, episodes, seconds)."""
    from oracle import oracle as orc
    from oracle import py_port

    torch.set_num_threads(1)
    pnet = py_port.PortNet({k: v.detach().cpu().numpy() for k, v in net_state.items()})
    np.random.seed(4)
    moves, eps_done = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        idx = int(start_state(eps_done))
        st = np.array([(idx // 3 ** (n_disks - 1 - d)) % 3 for d in range(n_disks)], np.uint8)
        ctr, active, done = 0, 1, 0
        mcts = py_port.PortMCTS(0.8, 0.25, S)  # one instance per game, as Muzero keeps one
        while not done and time.perf_counter() - t0 < seconds:
            obs = np.zeros(3 * n_disks)
            obs[np.arange(n_disks) * 3 + st] = 1.0
            action = mcts.run_mcts(obs, pnet, 1.0, False)[0]
            _, st, _, ctr, active, done, _ = orc.env_step(st, action, ctr, active, max_steps)
            moves += 1
        eps_done += 1
    return moves, eps_done, time.perf_counter() - t0


def cpu_baseline_solver(states, seconds):
    """hanoi_solver CPU baseline (tools/bench_eval.py): the C restatement (oracle/mzh_oracle.c) on
    one host core over a prefix of `states`.  Returns (moves of the prefix, states/s)."""
    from oracle import oracle as orc

    ref, k, t0 = [], 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and k < len(states):
        ref.append(orc.hanoi_solver(states[k]))
        k += 1
    return np.array(ref, np.int32), k / (time.perf_counter() - t0)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} != WORLD_SIZE {world}")
    ndev = torch.cuda.device_count()
    if a.dist_backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPUs (RCCL needs one GPU per rank)")
    gpu = local % ndev
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.dist_backend)

    from muzero_hanoi_amd import distributed as mdist
    from muzero_hanoi_amd import engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    N, S, B = a.disks, a.sims, a.roots_per_gpu
    GB = world * B  # global roots (weak scaling)
    torch.manual_seed(a.seed)
    net = MuZeroNet(3 * N, 6, 0.002, "cpu", TD_return=True)
    flat = engine.flat_weights(net.state_dict())
    if dist is not None:
        flat = mdist.broadcast_weights(flat, dev)  # weights broadcast once (~0.5 MB)
    eng = engine.Engine(N, S, B, 33, device=gpu)
    eng.load_weights(flat)

    # inputs for the GLOBAL batch in global root order, then this rank's contiguous shard
    sl = lambda x: mdist.shard(x, world, rank)
    obs = torch.from_numpy(sl(random_roots(N, GB, a.seed))).to(dev)
    noise, tie, u = rng.synthetic_draws(GB, deterministic=False, alpha=0.25, seed=a.seed)
    noise, tie, u = (torch.from_numpy(sl(x)).to(dev) for x in (noise, tie, u))
    out = eng.alloc_search_outputs(B, S)
    gather = dist is not None and not a.no_gather
    kern = None if a.kernel == "auto" else a.kernel
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, deterministic=False,
                   discount=0.8, eps=0.25, out=out, kernel=kern)
        if gather:
            return mdist.gather_visits(out["visits"], GB, world)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    # correctness sanity on the warmed-up result (outside timing)
    vis = out["visits"]
    assert int(vis.sum(1).min()) == S and int(vis.sum(1).max()) == S, "visit counts do not sum to n_sims"
    sel_mean = float(out["sel_steps"].double().mean()) / S

    # kernel-time probe: HIP events on the launch stream around each search launch
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        evs[k][0].record(stream)
        eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, deterministic=False,
                   discount=0.8, eps=0.25, out=out, kernel=kern)
        evs[k][1].record(stream)
        if gather:
            mdist.gather_visits(out["visits"], GB, world)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    if dist is not None:
        t = torch.tensor([dt, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kern_ms = float(t[0]), float(t[1])

    sims_total = world * B * S * a.steps
    value = sims_total / dt
    flops_launch = B * (S * MLP_FLOP_PER_SIM + root_flops(N))
    achieved = flops_launch / (kern_ms * 1e-3) / 1e12
    kern_sel = a.kernel if a.kernel != "auto" else ("wave" if B >= 53248 else "wave16" if B > 8192 else "coop")
    coop_rows = 32 if B > 4096 else 16  # mzh_api.hip choose_kernel() / pick_rows()
    kernel_name = {"wave": "mzh_wave_kernel<2,false,true>", "wave16": "mzh_wave_kernel<1,false,true>",
                   "coop": f"mzh_search_kernel<{coop_rows},false,*>"}[kern_sel]
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if tj.get("workload") == f"hanoi{N}_s{S}_roots{B}":
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    result = {
        "metric": "MCTS sims/sec (node) 4-disk Hanoi, 50 sims/move, 65k root batch; 1/2/4/8 GPU",
        "value": value,
        "unit": "sims/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: uniform random non-goal 4-disk root states, random-init MuZeroNet(TD_return=True)",
        "config": {"workload": f"hanoi{N}_s{S}_roots{B}_per_gpu" + (" (the metric's 65k-root batch on every GPU, weak scaling)"
                                                                   if B == 65536 else " (weak scaling)"),
                   "n_disks": N, "sims_per_move": S, "roots_per_gpu": B, "global_roots": world * B,
                   "parallelism": f"dp{world} (independent roots, all_gather of visits)" if world > 1 else "dp1"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": kernel_name, "kernel_ms": kern_ms,
                     "flop_per_launch": flops_launch, "sel_steps_per_sim": sel_mean},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(N, S, a.cpu_baseline_seconds, a.seed)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
