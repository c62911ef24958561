"""Benchmark: MCTS simulations/sec of the fused batched search (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]                       # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W             # N>1, one rank per GPU
    python bench.py --gpus N ...                                           # N>1 without a launcher:
        bench.py starts torch.distributed.run itself as a child process (before anything touches
        the GPU) and exits with its status, so the line always comes from N ranks

Workload (default): BASELINE.json's metric batch, 65,536 random non-goal 4-disk root states x 50
simulations, sharded contiguously over the N GPUs (strong scaling: 65,536 roots on 1 GPU, 8,192 per
GPU at N=8 = BASELINE configs[2] exactly).  `--config K` selects BASELINE configs[K] instead
(1: 4,096 roots S=50; 2: the default; 3: 16,384 roots S=200 N=4; 4: 262,144 roots S=100 N=7, sharded
over the ranks); `--roots-per-gpu B` runs B roots on every GPU (weak scaling, labelled so).
MuZeroNet(TD_return=True) with random-init weights (torch.manual_seed(0), broadcast once),
training-like search parameters (gamma 0.8, Dirichlet alpha 0.25 / eps 0.25, T=1, stochastic).
One step = one mzh_search launch over every root on the rank (root inference + S x {select, MFMA
MLP, backup} + play policy), followed by one RCCL all_gather of every root's result (visit
histogram, action, fp64 root Q: what run_mcts returns; north_star's only exchange).  Inputs are resident in HBM before timing starts.

Rank 0 prints ONE JSON line (contract in the task statement) including
  roofline        the fused search kernel (fp32-MFMA bound; achieved = algorithmic matmul FLOPs per
                  launch / mean launch time from HIP events on the launch stream);
  roofline.tree   select / expand / backup (HBM-bound): the same kernel's replay instantiation --
                  identical tree code with the network outputs read from HBM instead of computed --
                  timed live on the same roots; algorithmic tree bytes from the
                  kernel's own selection-step counts / its HIP-event time;
  cpu_baseline    the reference algorithm's Python restatement (oracle/py_port.py: object tree,
                  batch-1 torch-CPU MLP, NumPy RNG) as one process per host core over a bounded
                  sample (N=1 only), run before the GPU is touched.
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
# measured ceiling of back-to-back v_mfma_f32_16x16x4_f32 with distinct register operands, by waves per
# SIMD (tools/micro/lds_a_probe.hip, profiles/r02s2_mfma_ceiling.json): informational, beside the spec
# peak that `frac` is priced against
FP32_MFMA_MEASURED_TFLOPS = {1: 144.0, 2: 150.7}
HBM_PEAK_GBPS = 8000.0         # MI355X_MICROARCH.md: HBM3E peak (spec)
MLP_FLOP_PER_SIM = 203_776     # recurrent_inference matmul FLOPs (2 x 101,888 MAC)
# SURVEY.md 8d tree bytes: 124 B per selection step, 28 B per backed-up path node, 540 B per expansion
SEL_BYTES, BACKUP_BYTES, EXPAND_BYTES = 124, 28, 540
# the replay instantiation expands from recorded outputs: 32 B read (6 priors, value, reward) and the
# new child statistics written (6 priors + the leaf reward = 28 B); no latent is read or written
EXPAND_BYTES_REPLAY = 32 + 28

# one dependent 128-B tree-block load (an 8-lane group's slot reads, L2-resident footprint, one wave per
# SIMD on every CU): tools/micro/overlap_probe.hip, profiles/r04_overlap_probe.json -- the strict floor
TREE_LOAD_NS = 136.1
# loaded latency of a random 128-B line at the search kernels' concurrency (tools/micro/tree_mem_probe.hip,
# profiles/r05_tree_mem_probe.json: 2,048 waves, two per SIMD, each with W walks of dependent block loads,
# a lane pair per walk, uniformly random over F bytes): ns per dependent level by (footprint MB, walks per wave)
TREE_PROBE_NS = {(16, 1): 314.2, (16, 8): 368.4, (16, 32): 890.6,
                 (128, 1): 315.8, (128, 8): 375.8, (128, 32): 1216.2,
                 (448, 1): 316.6, (448, 8): 539.0, (448, 32): 1221.7,
                 (1344, 1): 317.4, (1344, 8): 589.4, (1344, 32): 1206.7}
# the same probe's random-line throughput with all 32 walks per wave streaming (no dependency), 448 MB footprint
TREE_RANDOM_LINE_GBPS = 6757.3

METRIC = "MCTS sims/sec (node) 4-disk Hanoi, 50 sims/move, 65k root batch; 1/2/4/8 GPU"
# BASELINE.json configs[1..4]: (disks, global roots, sims, description)
CONFIGS = {
    1: (4, 4096, 50, "BASELINE configs[1]: 4-disk, 4,096-root batch, 50 sims/move"),
    2: (4, 65536, 50, "BASELINE configs[2]: 4-disk, 65,536 roots, 50 sims/move, sharded over the GPUs"),
    3: (4, 16384, 200, "BASELINE configs[3]: 4-disk, 16,384 roots, 200 sims/move (deep tree)"),
    4: (7, 262144, 100, "BASELINE configs[4]: 7-disk, 262,144 roots, 100 sims/move, sharded over the GPUs"),
}


def root_flops(n_disks):
    return 2 * (768 * n_disks + 59_136)  # initial_inference matmul FLOPs


def launch_stats(ms):
    """per-launch HIP-event times -> min / median / max / mean; the line prices `frac` on the median so one
    slow or fast launch (in-run clock drift) does not move it"""
    a = np.asarray(ms, np.float64)
    return {"n": int(a.size), "min": float(a.min()), "median": float(np.median(a)), "max": float(a.max()),
            "mean": float(a.mean()), "argmax": int(a.argmax())}


def abba_order(rounds):
    """launch order of an A/B comparison taken in one window: A B B A per round, so neither leg always
    follows the other (the same clocks and the same predecessor mix for both)"""
    return [x for _ in range(rounds) for x in (0, 1, 1, 0)]


def ab_summary(ta, tb):
    """two legs timed in one ABBA window: each leg's launch_stats and the ratio of their medians"""
    sa, sb = launch_stats(ta), launch_stats(tb)
    return {"a": sa, "b": sb, "ratio_median": sb["median"] / sa["median"]}


def device_identity(dev):
    """what identifies this rank's GPU in a multi-GPU record: LOCAL_RANK, host, and the device's UUID / PCI
    location as torch reports them (fields torch does not have on this build are left out)"""
    import socket

    props = torch.cuda.get_device_properties(dev)
    ident = {"local_rank": int(os.environ.get("LOCAL_RANK", "0")), "host": socket.gethostname(),
             "device_index": dev.index, "name": props.name}
    for k in ("uuid", "pci_bus_id", "pci_device_id", "pci_domain_id"):
        v = getattr(props, k, None)
        if v is not None:
            ident[k] = str(v)
    return ident


def distinct_devices(idents):
    """physical GPUs among the ranks' identities: (host, UUID) when torch reports a UUID, else (host, PCI
    domain / bus / device), else (host, device index)"""
    keys = set()
    for d in idents:
        if "uuid" in d:
            keys.add((d["host"], d["uuid"]))
        elif "pci_bus_id" in d:
            keys.add((d["host"], d.get("pci_domain_id"), d["pci_bus_id"], d.get("pci_device_id")))
        else:
            keys.add((d["host"], d.get("device_index")))
    return len(keys)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", type=int, choices=sorted(CONFIGS), default=2,
                   help="BASELINE.json configs[K]; the global batch is sharded over the ranks (strong scaling)")
    p.add_argument("--roots-per-gpu", type=int, default=None,
                   help="weak scaling: this many roots on every GPU (overrides the config's global batch)")
    p.add_argument("--shard", default=None, metavar="R/W",
                   help="run rank R's shard of the config's global batch for a W-GPU job, alone on this GPU "
                        "(the per-GPU work of the W-GPU bench, same roots and draws; value = this GPU's sims/s)")
    p.add_argument("--sims", type=int, default=None)
    p.add_argument("--disks", type=int, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-gather", action="store_true")
    p.add_argument("--overlap-gather", action="store_true",
                   help="N > 1, even shards: run each step's all_gather asynchronously on the backend's stream "
                        "beside the next step's search (default: on the launch stream after its search; with "
                        "gloo on one GPU the overlapped form measured slower, 17.4 vs 11.9 ms per step, and "
                        "RCCL's is unmeasured: one GPU per call here)")
    p.add_argument("--no-tree", action="store_true", help="skip the live select/backup (replay) measurement")
    p.add_argument("--no-minmax-leg", action="store_true",
                   help="skip timing the instantiation searches with caller MinMaxStats bounds run (training / acting)")
    p.add_argument("--kernel", choices=["auto", "coop", "occ2", "wave", "wave16"], default="auto")
    p.add_argument("--tile", type=int, choices=[16, 32], default=None,
                   help="cooperative kernel: roots per workgroup (default by batch size)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, one rank per GPU); gloo lets ranks share a GPU to rehearse the N>1 path")
    p.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    p.add_argument("--cpu-baseline-procs", type=int, default=0,
                   help="0: one process per physical core, capped at the GPU box's 16-CPU share per job")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    p.add_argument("--dry-run", action="store_true",
                   help="rank plumbing only: start the ranks, form the process group, print the line's n_gpus / "
                        "dist / shard fields without touching a GPU (tests/test_bench_cpu.py, gloo)")
    return p.parse_args()


def relaunch_with_ranks(n):
    """`--gpus N` (N > 1) started without a launcher: run the same command under
    torch.distributed.run with N local ranks as a CHILD process (this process has not initialised
    the GPU: no exec after a HIP call) and return its exit status"""
    import socket
    import subprocess

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: --gpus {n} without a launcher; starting {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return subprocess.run(cmd).returncode


def random_roots(n_disks, B, seed):
    """uniform over the 3^N states excluding the goal (env/hanoi.py:103-109 distribution)"""
    g = np.random.default_rng(seed)
    goal = 3 ** n_disks - 1
    idx = g.integers(0, goal, size=B)  # [0, goal) == every state but the goal (index 3^N - 1)
    st = np.stack([(idx // 3 ** (n_disks - 1 - d)) % 3 for d in range(n_disks)], 1)
    obs = np.zeros((B, 3 * n_disks), np.float32)
    obs[np.arange(B)[:, None], np.arange(n_disks) * 3 + st] = 1.0
    return obs


# ------------------------------------------------------------------------------------------------
# CPU baseline: the reference algorithm (oracle/py_port.py restates MCTS/mcts.py:34-126 + node.py +
# networks.py and matches the reference's visit counts bit for bit) on the host cores.
# ------------------------------------------------------------------------------------------------
def _cpu_worker(args):
    """one host process: fresh MCTS per root over roots k, k + P, k + 2P, ... for `seconds`"""
    n_disks, S, seconds, seed, k, P = args
    torch.set_num_threads(1)
    from muzero_hanoi_amd.networks import MuZeroNet
    from oracle import py_port

    torch.manual_seed(seed)
    net = MuZeroNet(3 * n_disks, 6, 0.002, "cpu", TD_return=True)
    pnet = py_port.PortNet({kk: v.numpy() for kk, v in net.state_dict().items()})
    obs = random_roots(n_disks, 4096, seed + 99).astype(np.float64)
    np.random.seed(seed + k)
    roots = 0
    t0 = time.perf_counter()
    r = k
    while time.perf_counter() - t0 < seconds:
        m = py_port.PortMCTS(0.8, 0.25, S)
        m.run_mcts(obs[r % len(obs)], pnet, 1.0, False)
        roots += 1
        r += P
    return roots, time.perf_counter() - t0


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _physical_cores(cpus):
    """distinct (package, core) pairs among the logical CPUs `cpus` (SMT siblings counted once)"""
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            seen.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            seen.add(("?", str(c)))
    return len(seen)


# the GPU box grants one job a 16-CPU share of its host (os.cpu_count() shows the whole machine): the
# measured pool stays within it; the all-physical-core figure BASELINE.md 3 names is reported beside
# it as the single-process rate x the physical cores (linear scaling, an upper bound)
CPU_SHARE = 16


def cpu_baseline(n_disks, S, seconds, seed, procs=0):
    """One process per core of the job's CPU share (torch.set_num_threads(1) each, roots partitioned
    round-robin), aggregate sims/s = all processes' sims / the slowest process's wall time; plus the
    1-process figure from a separate single-process run, and that figure scaled to every physical
    core of the affinity set (BASELINE.md 3's "one process per physical host core"), labelled as an
    extrapolation."""
    import multiprocessing as mp

    aff = sorted(os.sched_getaffinity(0))
    avail = len(aff)
    phys = _physical_cores(aff)
    P = procs if procs > 0 else min(phys, CPU_SHARE)
    ctx = mp.get_context("spawn")  # fresh interpreters; this process has not touched the GPU
    single_roots, single_dt = _cpu_worker((n_disks, S, seconds / 3, seed, 0, 1))
    with ctx.Pool(P) as pool:
        res = pool.map(_cpu_worker, [(n_disks, S, seconds, seed, k, P) for k in range(P)])
    roots = sum(r for r, _ in res)
    dt = max(t for _, t in res)
    single = single_roots * S / single_dt
    return {"value": roots * S / dt, "unit": "sims/s", "cores": P, "kind": "port",
            "cpu_model": _cpu_model(), "cores_available": avail, "physical_cores_available": phys,
            "single_core_value": single,
            "all_physical_cores": {"value": single * phys, "cores": phys, "measured": False,
                                   "what": f"single_core_value x {phys} physical cores of the affinity set "
                                           f"(BASELINE.md 3: one process per physical host core), linear scaling "
                                           f"assumed -- an upper bound; not measured because the GPU box grants "
                                           f"this job a {CPU_SHARE}-CPU share and a {phys}-process pool would "
                                           f"oversubscribe it (the measured {P}-process value scales "
                                           f"{roots * S / dt / max(single, 1e-9):.1f}x over one process)"},
            "sample": f"{P} processes x {seconds:.0f} s (one per core of the job's CPU share, torch threads=1 each): {roots} roots x "
                      f"{S} sims, {n_disks}-disk, fresh MCTS per root, T=1 stochastic, roots partitioned "
                      f"round-robin; single_core_value: 1 process, {single_roots} roots in {single_dt:.1f} s. "
                      f"oracle/py_port.py restates MCTS/mcts.py + networks.py and matches the reference's "
                      f"visits bit-exactly"}


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


def tree_bytes(sel_steps_sum, n_roots, S, expand_bytes):
    """SURVEY.md 8d algorithmic tree bytes: 124 per selection step, 28 per backed-up node (each
    simulation backs up its d selected path nodes + the root), expand_bytes per expansion"""
    return SEL_BYTES * sel_steps_sum + BACKUP_BYTES * (sel_steps_sum + n_roots * S) + expand_bytes * n_roots * S


def search_plan(S, B, kern="auto", tile=None, replay=False, minmax_in=False, support=33):
    """the launch plan libmzh reports for this workload (mzh_search_plan_query: the same host code
    that picks the instantiation mzh_search launches -- kernel, tile, template arguments)"""
    from muzero_hanoi_amd import _lib, engine

    return _lib.search_plan(support, B, S, engine.search_flags(None if kern == "auto" else kern, tile),
                            replay=replay, minmax_in=minmax_in)


def traffic_key(n_disks, S, B, kern="auto", tile=None, minmax_in=False):
    """the key of one bench workload in profiles/traffic_latest.json (tools/traffic.py writes it
    from the same function): disks, sims, roots on this GPU and the fused kernel instantiation the
    library launches for them"""
    k = search_plan(S, B, kern, tile, minmax_in=minmax_in)["kernel"].replace(" ", "")
    return f"hanoi{n_disks}_s{S}_roots{B}_{k}"


def workload_shape(config, world=1, rank=0, roots_per_gpu=None, disks=None, sims=None):
    """(disks, sims, roots on this rank, global roots) of a bench invocation"""
    from muzero_hanoi_amd import distributed as mdist

    N, GB, S, _ = CONFIGS[config]
    N, S = disks or N, sims or S
    if roots_per_gpu is not None:
        GB = world * roots_per_gpu
    s0, s1 = mdist.shard_range(GB, world, rank)
    return N, S, s1 - s0, GB


def lookup_traffic(path, key):
    """(entry, note): the PMC-counted HBM bytes of this workload if profiled on THIS build"""
    if not os.path.exists(path):
        return None, "no traffic file"
    try:
        entries = json.load(open(path)).get("entries", {})
    except Exception as e:  # noqa: BLE001
        return None, f"unreadable traffic file: {e}"
    ent = entries.get(key)
    if ent is None:
        return None, f"workload {key} not profiled"
    from muzero_hanoi_amd import _lib

    if ent.get("build_id") != _lib.build_id():
        return None, f"profiled on build {ent.get('build_id')}, not this build {_lib.build_id()}"
    return ent, "rocprofv3 PMC of this build (tools/prof.sh + tools/traffic.py)"


def probe_latency_ns(footprint_mb, walks_per_wave):
    """TREE_PROBE_NS interpolated: log-linear in the footprint, linear in the walks per wave (clamped)"""
    fps = sorted({f for f, _ in TREE_PROBE_NS})
    ws = sorted({w for _, w in TREE_PROBE_NS})
    f = min(max(footprint_mb, fps[0]), fps[-1])
    w = min(max(walks_per_wave, ws[0]), ws[-1])

    def lerp(xs, x, fn, log=False):
        for a, b in zip(xs, xs[1:]):
            if a <= x <= b:
                t = (np.log(x) - np.log(a)) / (np.log(b) - np.log(a)) if log else (x - a) / (b - a)
                return fn(a) * (1 - t) + fn(b) * t
        return fn(xs[-1])

    return lerp(fps, f, lambda ff: lerp(ws, w, lambda ww: TREE_PROBE_NS[(ff, ww)]), log=True)


def tree_latency_model(levels, S, plan, B, kernel_ms=None):
    """The select / backup latency ceiling from the kernel's own count: every lockstep group (a wave of
    the wave kernel, a workgroup of the cooperative kernels) waits, simulation after simulation, for its
    deepest root's dependent tree-block loads -- `levels[g]` of them in all (mzh_search_args.lockstep_levels).
    The groups of one round run concurrently, so the launch takes at least max_g levels[g] x the latency
    of one such load.  Priced twice: `floor_ms` with the L2-resident latency (a strict lower bound) and
    `model_ms` with the probe's loaded latency of a random 128-B line at this launch's footprint and
    walks per wave (TREE_PROBE_NS) -- the latency the levels actually see when every group walks at once."""
    lv = np.asarray(levels, np.float64)
    g = plan["roots_per_wave"] if plan["wave"] else plan["roots_per_workgroup"]
    n = -(-B // g)
    lv = lv[:n]
    slots = lockstep_slots(plan)
    rounds = -(-n // slots)
    deepest = float(lv.max()) if rounds == 1 else float(rounds * lv.mean())
    walks = plan["roots_per_wave"]  # walks in flight per wave: its roots (cooperative: R / 4 per wave)
    footprint_mb = B * (S + 1) * 128 / 2 ** 20
    lat = probe_latency_ns(footprint_mb, walks)
    out = {"groups": n, "roots_per_group": g, "rounds": rounds,
           "levels_per_sim": {"mean_group": float(lv.mean()) / S, "max_group": float(lv.max()) / S},
           "floor_ms": deepest * TREE_LOAD_NS * 1e-6, "floor_load_ns": TREE_LOAD_NS,
           "model_ms": deepest * lat * 1e-6, "model_load_ns": lat,
           "model_probe": {"footprint_mb": footprint_mb, "walks_per_wave": walks,
                           "source": "tools/micro/tree_mem_probe.hip, profiles/r05_tree_mem_probe.json"}}
    if kernel_ms:
        out["floor_frac"] = out["floor_ms"] / kernel_ms
        out["frac"] = out["model_ms"] / kernel_ms
    return out


CUS = 256                  # MI355X: 8 XCDs x 32 CUs
LDS_PER_CU = 160 * 1024    # bytes


def workgroups_per_cu(plan):
    """co-resident workgroups per CU for a plan: its LDS footprint and its register budget -- the
    wave kernel is built __launch_bounds__(256, 2) (<= 256 VGPRs: two waves per SIMD), the cooperative
    kernel __launch_bounds__(256, 1) (one wave per SIMD); both use 4-wave workgroups"""
    waves_per_simd_max = 2 if plan["wave"] else 1
    by_lds = LDS_PER_CU // max(1, int(plan["smem_bytes"]))
    by_regs = waves_per_simd_max * 4 // max(1, int(plan["threads_per_workgroup"]) // 64)
    return max(1, min(by_lds, by_regs))


def lockstep_slots(plan):
    """lockstep groups the GPU runs at once: the wave kernel's waves (each a group of 16 NT roots),
    the cooperative kernel's workgroups (each a group of R roots)"""
    wg = CUS * workgroups_per_cu(plan)
    return wg * (int(plan["threads_per_workgroup"]) // 64) if plan["wave"] else wg


def waves_per_simd(plan, B):
    """waves sharing a SIMD: the wave kernel runs B / roots_per_wave waves, two 4-wave workgroups per
    CU at most (1,024 SIMDs); the cooperative kernel one 4-wave workgroup per CU"""
    if not plan["wave"]:
        return 1
    waves = -(-B // plan["roots_per_wave"])
    return min(2, max(1, -(-waves // 1024)))


def main():
    a = parse()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(relaunch_with_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} != WORLD_SIZE {world}: the line would not describe the ranks that ran")
    N, GB, S, desc = CONFIGS[a.config]
    N = a.disks or N
    S = a.sims or S
    weak = a.roots_per_gpu is not None
    if weak:
        GB = world * a.roots_per_gpu
    # --shard R/W: this process plays rank R of a W-GPU job (one GPU, no collective)
    srank, sworld = (rank, world) if a.shard is None else map(int, a.shard.split("/"))
    if a.shard is not None and (world > 1 or weak or not 0 <= srank < sworld):
        raise SystemExit("--shard R/W needs one process, no --roots-per-gpu, and 0 <= R < W")
    if GB < max(world, sworld):
        raise SystemExit(f"{GB} roots cannot give each of {max(world, sworld)} ranks a non-empty shard")
    if a.dry_run:
        return dry_run(a, world, rank, GB, S, N)

    # CPU baseline first (rank 0, N=1): spawned host processes, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(N, S, a.cpu_baseline_seconds, a.seed, a.cpu_baseline_procs)

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

    from muzero_hanoi_amd import _lib
    from muzero_hanoi_amd import distributed as mdist
    from muzero_hanoi_amd import engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    s0, s1 = mdist.shard_range(GB, sworld, srank)
    B = s1 - s0  # this rank's roots
    torch.manual_seed(a.seed)
    net = MuZeroNet(3 * N, 6, 0.002, "cpu", TD_return=True)
    flat = engine.flat_weights(net.state_dict())
    if dist is not None:
        flat = mdist.broadcast_weights(flat, dev)  # weights broadcast once (~0.5 MB)
    eng = engine.Engine(N, S, B, 33, device=gpu)
    eng.load_weights(flat)

    # inputs for the GLOBAL batch in global root order, then this rank's contiguous shard
    sl = lambda x: mdist.shard(x, sworld, srank)
    obs = torch.from_numpy(sl(random_roots(N, GB, a.seed))).to(dev)
    # the reference's draws (Dirichlet noise, first-tie choice, action uniform) for the GLOBAL batch in
    # reference order: what GB sequential run_mcts calls after np.random.seed(seed) consume
    # (rng.predraw, libmzh's host restatement of NumPy's legacy stream), timed as host set-up
    t_pd = time.perf_counter()
    noise, tie, u = rng.predraw(GB, deterministic=False, alpha=0.25, rng=np.random.RandomState(a.seed))
    predraw_ms = (time.perf_counter() - t_pd) * 1e3
    noise, tie, u = (torch.from_numpy(sl(x)).to(dev) for x in (noise, tie, u))
    out = eng.alloc_search_outputs(B, S)
    gather = dist is not None and not a.no_gather
    kern = None if a.kernel == "auto" else a.kernel
    stream = torch.cuda.current_stream(dev)

    def search():
        eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, deterministic=False,
                   discount=0.8, eps=0.25, out=out, kernel=kern, tile=a.tile)

    # one launch, its correctness sanity and the kernel-time probe's set-up first, then the warm-up launches
    # straight into the timed ones: host work between them would idle the GPU (its clocks drop, and the first
    # timed launch paid ~1.1 ms for it -- profiles/r06_bench_first_launch.json)
    search()
    if gather:
        mdist.gather_results(out, GB, world)
    torch.cuda.synchronize(dev)
    vis = out["visits"]
    assert int(vis.sum(1).min()) == S and int(vis.sum(1).max()) == S, "visit counts do not sum to n_sims"
    sel_sum = float(out["sel_steps"].double().sum())
    # kernel-time probe: HIP events on the launch stream around each search launch
    plan = search_plan(S, B, a.kernel, a.tile)
    assert out["_plan"]["kernel"] == plan["kernel"], (out["_plan"], plan)  # the query names what launched
    if a.kernel == "occ2":
        assert plan["kernel"].startswith("mzh_search_occ2_kernel<"), plan  # --kernel occ2 measures occ2
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    gevs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    for _ in range(a.warmup):
        search()
        if gather:
            mdist.gather_results(out, GB, world)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    overlap = gather and a.overlap_gather and GB % world == 0
    t0 = time.perf_counter()
    pend = []
    for k in range(a.steps):
        evs[k][0].record(stream)
        search()
        evs[k][1].record(stream)
        if overlap:  # step k's results gathered beside step k+1's search (both inside the timed region)
            pend.append(mdist.gather_results_async(out, GB, world))
        elif gather:
            mdist.gather_results(out, GB, world)
            gevs[k].record(stream)
    for w in pend:
        w[0].wait()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    kstats = launch_stats([s.elapsed_time(e) for s, e in evs])
    kern_ms = kstats["median"]
    gather_ms = None
    if overlap:
        # what one gather costs on its own (untimed probe after the loop: HIP events around a synchronous one)
        gp = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for s_, e_ in gp:
            s_.record(stream)
            mdist.gather_results(out, GB, world)
            e_.record(stream)
        torch.cuda.synchronize(dev)
        gather_ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in gp]))
    elif gather:
        gather_ms = float(np.mean([evs[k][1].elapsed_time(gevs[k]) for k in range(a.steps)]))

    # the instantiation training and acting searches run: the same roots with caller-given MinMaxStats
    # bounds (run_mcts passes the MCTS instance's persistent bounds; fresh ones here), timed apart
    mm = None
    if not a.no_minmax_leg:
        mm_in = torch.tensor([[-np.inf, np.inf]], dtype=torch.float64, device=dev).expand(B, 2).contiguous()
        mout = eng.alloc_search_outputs(B, S)

        def search_mm():
            eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, minmax_in=mm_in, temperature=1.0,
                       deterministic=False, discount=0.8, eps=0.25, out=mout, kernel=kern, tile=a.tile)

        search_mm()
        torch.cuda.synchronize(dev)
        assert torch.equal(mout["visits"], out["visits"]), "fresh caller bounds changed the search"
        # A B B A with the plain search in one window, so both legs see the same clocks and neither always
        # runs after the other (round 5's 5 alternated pairs read the plain kernel 3% slower than the
        # 20-step loop: a drift artefact in the ratio)
        order = abba_order(4)
        mev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in order]
        for leg, (s_, e_) in zip(order, mev):
            s_.record(stream)
            (search, search_mm)[leg]()
            e_.record(stream)
        torch.cuda.synchronize(dev)
        legs = ([], [])
        for leg, (s_, e_) in zip(order, mev):
            legs[leg].append(s_.elapsed_time(e_))
        ab = ab_summary(*legs)
        mm = {"kernel": mout["_plan"]["kernel"], "kernel_ms": ab["b"]["median"],
              "plain_kernel_ms_same_window": ab["a"]["median"], "ratio": ab["ratio_median"],
              "launch_stats": ab["b"], "plain_launch_stats": ab["a"],
              "what": "the same search with minmax_in given (fresh bounds: identical visits), the instantiation "
                      "MCTS.run_mcts and batched self-play launch; 8 launches interleaved A B B A with 8 plain ones "
                      "in one window, HIP events, medians"}

    # select / expand / backup alone: the replay instantiation of the same kernel on the same roots,
    # network outputs drawn like a random-init network's (near-uniform priors, small values)
    tree = None
    if not a.no_tree:
        g = np.random.default_rng(a.seed + 7)
        rp = dict(root_pi=torch.from_numpy(g.dirichlet(np.full(6, 20.0), size=B).astype(np.float32)).to(dev),
                  pi=torch.from_numpy(g.dirichlet(np.full(6, 20.0), size=(B, S)).astype(np.float32)).to(dev),
                  reward=torch.from_numpy(g.normal(0, 0.05, (B, S)).astype(np.float32)).to(dev),
                  value=torch.from_numpy(g.normal(0, 0.5, (B, S)).astype(np.float32)).to(dev))
        # the kernel's simulation-major replay records, packed once before timing (engine.pack_replay)
        rp = dict(root_pi=rp["root_pi"], sim=engine.pack_replay(rp))
        rout = eng.alloc_search_outputs(B, S)

        def replay():
            eng.search(S, replay=rp, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, deterministic=False,
                       discount=0.8, eps=0.25, out=rout, kernel=kern, tile=a.tile)

        # one untimed launch also counts each lockstep group's selection levels (the latency model's input;
        # the timed launches below do not count, so the count costs them nothing)
        lout = eng.alloc_search_outputs(B, S, lockstep=True)
        eng.search(S, replay=rp, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, deterministic=False,
                   discount=0.8, eps=0.25, out=lout, kernel=kern, tile=a.tile)
        replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(lout["visits"], rout["visits"]), "the level count changed the search"
        levels = lout["lockstep_levels"].cpu().numpy()
        rsel = float(rout["sel_steps"].double().sum())
        tev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for s_, e_ in tev:
            s_.record(stream)
            replay()
            e_.record(stream)
        torch.cuda.synchronize(dev)
        tstats = launch_stats([s_.elapsed_time(e_) for s_, e_ in tev])
        tree_ms = tstats["median"]
        tb = tree_bytes(rsel, B, S, EXPAND_BYTES_REPLAY)
        tree = {"bound": "hbm", "kernel": rout["_plan"]["kernel"],
                "bytes_per_launch": tb, "kernel_ms": tree_ms, "launch_stats": tstats,
                "achieved": tb / (tree_ms * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "sel_steps_per_sim": rsel / (B * S),
                "frac": tb / (tree_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, "traffic": None,
                "fused_tree_bytes_per_launch": tree_bytes(sel_sum, B, S, EXPAND_BYTES),
                "random_line": {"ceiling_gbps": TREE_RANDOM_LINE_GBPS,
                                "frac": tb / (tree_ms * 1e-3) / 1e9 / TREE_RANDOM_LINE_GBPS,
                                "what": "the same bytes against the random 128-B line throughput the probe measured "
                                        "at this concurrency (tools/micro/tree_mem_probe.hip), not the streaming peak"},
                "latency": tree_latency_model(levels, S, rout["_plan"], B, tree_ms),
                "what": "select/expand/backup only: the search kernel's replay instantiation (same tree code, "
                        "network outputs read from HBM), same roots and draws; bytes = SURVEY.md 8d (124 B per "
                        "selection step, 28 B per backed-up node, 60 B per replayed expansion) with the kernel's "
                        "own selection-step count; fused_tree_bytes_per_launch: the same count in the fused "
                        "search (540 B per expansion incl. the latent read/write)"}

    if tree is not None:
        tree["latency"]["what"] = ("fraction of the tree kernel's HIP-event time that its lockstep groups' dependent "
                                   "block loads take in sequence (kernel-counted levels x the probe's loaded "
                                   "latency; floor_frac with the L2-resident latency), bench.tree_latency_model")
        fr = {"hbm": tree["frac"], "random_line": tree["random_line"]["frac"], "latency": tree["latency"]["frac"]}
        tree["binding"] = {"ceiling": max(fr, key=fr.get), "frac": max(fr.values()), "fracs": fr}
    dinfo = None
    if dist is not None:
        # every rank's own figures, gathered (so a scaling record shows the ranks RCCL saw), then maxed
        mine = torch.tensor([dt, kern_ms, tree["kernel_ms"] if tree else 0.0, gather_ms or 0.0, float(B)],
                            dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
        dist.all_gather(allr, mine)
        allr = torch.stack(allr).cpu().numpy()
        idents = [None] * dist.get_world_size()
        dist.all_gather_object(idents, dict(device_identity(dev), rank=rank))
        dinfo = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                 "devices": idents, "distinct_devices": distinct_devices(idents),
                 "gather_ms_per_step": {"max": float(allr[:, 3].max()), "min": float(allr[:, 3].min())} if gather else None,
                 "kernel_ms_per_rank": [float(x) for x in allr[:, 1]],
                 "roots_per_rank": [int(x) for x in allr[:, 4]],
                 "step_wall_s_per_rank": [float(x) for x in allr[:, 0]],
                 "gather_overlapped": bool(overlap),
                 "what": "one process per rank; gather = the all_gather of every root's visits/action/root Q "
                         "(HIP events around a synchronous one on the launch stream, mean); with "
                         "gather_overlapped each step's gather runs on the backend's stream beside the next "
                         "step's search and the timed region ends after the last one completes"}
        t = torch.tensor(allr.max(0), dtype=torch.float64)
        dt, kern_ms = float(t[0]), float(t[1])
        if tree:
            tree["kernel_ms"] = float(t[2])
            tree["achieved"] = tree["bytes_per_launch"] / (tree["kernel_ms"] * 1e-3) / 1e9
            tree["frac"] = tree["achieved"] / HBM_PEAK_GBPS
            tree["random_line"]["frac"] = tree["achieved"] / TREE_RANDOM_LINE_GBPS
            tree["latency"]["frac"] = tree["latency"]["model_ms"] / tree["kernel_ms"]
            tree["latency"]["floor_frac"] = tree["latency"]["floor_ms"] / tree["kernel_ms"]
            fr = {"hbm": tree["frac"], "random_line": tree["random_line"]["frac"], "latency": tree["latency"]["frac"]}
            tree["binding"] = {"ceiling": max(fr, key=fr.get), "frac": max(fr.values()), "fracs": fr}

    sims_total = (GB if a.shard is None else B) * S * a.steps
    value = sims_total / dt
    flops_launch = B * (S * MLP_FLOP_PER_SIM + root_flops(N))
    achieved = flops_launch / (kern_ms * 1e-3) / 1e12
    kname = plan["kernel"]
    wps = waves_per_simd(plan, B)
    tkey = traffic_key(N, S, B, a.kernel, a.tile)
    if mm is not None:
        mm["frac"] = flops_launch / (mm["kernel_ms"] * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS
    tent, tnote = lookup_traffic(a.traffic_json, tkey)
    traffic = tent.get("hbm_bytes_per_launch") if tent else None
    if tree is not None and tent:
        tree["traffic"] = tent.get("tree_hbm_bytes_per_launch")
        if tent.get("tree_issue_frac") is not None:
            # the issue ceiling: the fraction of the SIMDs' cycles some wave issued (PMC of this build)
            twps = waves_per_simd(rout["_plan"], B)
            tree["issue"] = {"frac": tent["tree_issue_frac"], "waitcnt_frac": tent.get("tree_waitcnt_frac"),
                             "waves_per_simd": twps, "upper_bound": twps > 1,
                             "note": "SQ_ACTIVE_INST_ANY sums per-wave issue cycles over waves: with two waves per "
                                     "SIMD their overlapping issue is counted twice, so frac is an upper bound of "
                                     "the SIMDs' issue-busy fraction there" if twps > 1 else
                                     "one wave per SIMD: the SIMDs' issue-busy fraction",
                             "source": "rocprofv3 --pmc SQ_ACTIVE_INST_ANY x 4 / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8) "
                                       "of this build (tools/prof.sh + tools/traffic.py)"}
            tree["binding"]["fracs"]["issue"] = tent["tree_issue_frac"]
            b = tree["binding"]["fracs"]
            tree["binding"].update(ceiling=max(b, key=b.get), frac=max(b.values()))

    if weak:
        workload = (f"weak scaling: {N}-disk, {B} roots per GPU ({GB} over {world} GPUs), {S} sims/move "
                    f"(not a BASELINE config unless N x roots matches one)")
    elif a.shard is not None:
        workload = (desc + f": rank {srank}'s shard of an N={sworld} job ({B} roots), run alone on one GPU "
                    f"(value = this GPU's sims/s; the N={sworld} job's per-GPU work)")
    else:
        workload = desc + (f": {B} roots per GPU at N={world}" if world > 1 else
                           (" (the whole batch on one GPU)" if a.config in (2, 4) else ""))
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "sims/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic: uniform random non-goal {N}-disk root states, random-init MuZeroNet(TD_return=True)",
        "config": {"workload": workload, "baseline_config": None if weak else a.config, "n_disks": N,
                   "sims_per_move": S, "roots_per_gpu": B, "global_roots": GB, "shard": a.shard,
                   "parallelism": f"dp{world} (independent roots, all_gather of visits/action/root Q)" if world > 1 else "dp1"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": {"key": tkey, "note": tnote,
                                        "kernel_avg_ns_profiled": tent.get("avg_ns") if tent else None},
                     "kernel": kname, "kernel_ms": kern_ms, "launch_stats": kstats,
                     "kernel_ms_what": "median of the timed launches' HIP-event times (this rank; max over ranks "
                                       "at N > 1); achieved and frac are priced on it",
                     "flop_per_launch": flops_launch, "sel_steps_per_sim": sel_sum / (B * S),
                     "measured_ceiling": {"value": FP32_MFMA_MEASURED_TFLOPS[wps],
                                          "frac": achieved / FP32_MFMA_MEASURED_TFLOPS[wps],
                                          "waves_per_simd": wps,
                                          "what": "back-to-back MFMAs with distinct register operands at this "
                                                  "kernel's waves per SIMD (tools/micro/lds_a_probe.hip); "
                                                  "informational -- frac above is against the spec peak"},
                     "plan": plan, "with_minmax_in": mm, "tree": tree},
        "cpu_baseline": cpu,
        "predraw": {"ms": predraw_ms, "roots": GB, "search_kernel_ms": kern_ms, "ratio_to_search": predraw_ms / kern_ms,
                    "what": "host set-up, outside the timed region: the reference-order draws of all global roots "
                            "(Dirichlet(0.25) noise, first-tie choice, action uniform; MCTS/mcts.py:57-66,149, "
                            "MCTS/node.py:86, MCTS/mcts.py:118-120) on NumPy's legacy MT19937 stream by "
                            "rng.predraw (libmzh mzh_rng_predraw), bit-identical to the NumPy calls"},
        "dist": dinfo,
        "build_id": _lib.build_id(),
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def dry_run(a, world, rank, GB, S, N):
    """--dry-run: the ranks and the process group, no GPU (rank 0 prints the line's rank fields)"""
    from muzero_hanoi_amd import distributed as mdist

    shards = [mdist.shard_range(GB, world, r) for r in range(world)]
    dinfo = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(a.dist_backend)
        import socket

        mine = torch.tensor([float(rank), float(shards[rank][1] - shards[rank][0])], dtype=torch.float64)
        allr = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
        dist.all_gather(allr, mine)
        idents = [None] * dist.get_world_size()
        dist.all_gather_object(idents, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                                        "host": socket.gethostname()})
        dinfo = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                 "ranks": [int(x[0]) for x in allr], "roots_per_rank": [int(x[1]) for x in allr],
                 "devices": idents}
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "config": {"baseline_config": a.config, "n_disks": N, "sims_per_move": S,
                                     "global_roots": GB, "shards": shards},
                          "dist": dinfo}), flush=True)


if __name__ == "__main__":
    main()
