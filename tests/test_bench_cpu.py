"""bench.py host logic on CPU: the workload keys shared with tools/traffic.py, the build-id gate
on the PMC traffic it reports, and the CPU-baseline core accounting."""
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_committed_traffic_has_the_default_bench_key():
    """profiles/traffic_latest.json holds an entry under the exact key the driver's default bench
    command (configs[2] on one GPU) looks up"""
    import bench

    key = bench.traffic_key(*bench.workload_shape(2)[:3])
    assert key == "hanoi4_s50_roots65536_mzh_wave_kernel<2,false,true>"
    doc = json.load(open(os.path.join(ROOT, "profiles", "traffic_latest.json")))
    assert key in doc["entries"]
    ent = doc["entries"][key]
    assert ent["hbm_bytes_per_launch"] > 0 and ent["tree_hbm_bytes_per_launch"] > 0 and ent["build_id"]


def test_traffic_keys_of_every_config_and_shard():
    """the key names the fused instantiation the library's plan query reports -- the same host code
    mzh_search launches from -- for every BASELINE config and per-GPU shard the driver runs"""
    import bench

    wave, wave16 = "mzh_wave_kernel<2,false,true>", "mzh_wave_kernel<1,false,true>"
    c32, c16 = "mzh_search_kernel<32,false,true,true,false>", "mzh_search_kernel<16,false,true,true,false>"
    want = {(1, 1): f"hanoi4_s50_roots4096_{c16}", (1, 2): f"hanoi4_s50_roots2048_{c16}",
            (2, 1): f"hanoi4_s50_roots65536_{wave}", (2, 2): f"hanoi4_s50_roots32768_{wave16}",
            (2, 4): f"hanoi4_s50_roots16384_{wave16}", (2, 8): f"hanoi4_s50_roots8192_{c32}",
            (3, 1): f"hanoi4_s200_roots16384_{wave16}", (3, 2): f"hanoi4_s200_roots8192_{c16}",
            (4, 1): f"hanoi7_s100_roots262144_{wave}", (4, 4): f"hanoi7_s100_roots65536_{wave}",
            (4, 8): f"hanoi7_s100_roots32768_{wave16}"}
    for (cfg, world), key in want.items():
        for rank in range(world):
            N, S, B, _ = bench.workload_shape(cfg, world=world, rank=rank)
            assert bench.traffic_key(N, S, B) == key, (cfg, world, rank)
    # a forced tile is part of the key (its PMC entry is not the default tile's)
    assert bench.traffic_key(4, 50, 8192, tile=16) == f"hanoi4_s50_roots8192_{c16}"
    assert bench.traffic_key(4, 50, 8192, minmax_in=True) == f"hanoi4_s50_roots8192_{c32[:-7]},true>"


def test_bench_plan_is_the_library_plan():
    """bench reports the library's plan (kernel, waves per SIMD) for every config x shard"""
    import bench

    from muzero_hanoi_amd import _lib

    for cfg in (1, 2, 3, 4):
        for world in (1, 2, 4, 8):
            N, S, B, _ = bench.workload_shape(cfg, world=world)
            pl = bench.search_plan(S, B)
            assert pl == _lib.search_plan(33, B, S)
            assert bench.waves_per_simd(pl, B) in (1, 2)
            if pl["wave"] and pl["roots_per_wave"] == 32 and B >= 65536:
                assert bench.waves_per_simd(pl, B) == 2


def test_traffic_is_reported_only_for_the_profiled_build(tmp_path):
    import bench

    from muzero_hanoi_amd import _lib, build

    build.build()
    key = "hanoi4_s50_roots65536_mzh_wave_kernel<2,false,true>"
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"entries": {key: {"build_id": "0" * 20, "hbm_bytes_per_launch": 1.0}}}))
    ent, note = bench.lookup_traffic(str(p), key)
    assert ent is None and "not this build" in note
    p.write_text(json.dumps({"entries": {key: {"build_id": _lib.build_id(), "hbm_bytes_per_launch": 1.0}}}))
    ent, note = bench.lookup_traffic(str(p), key)
    assert ent["hbm_bytes_per_launch"] == 1.0
    assert bench.lookup_traffic(str(p), "other")[0] is None


def test_physical_core_count():
    import bench

    cpus = sorted(os.sched_getaffinity(0))
    n = bench._physical_cores(cpus)
    assert 1 <= n <= len(cpus)


def test_tree_latency_model():
    """the select/backup latency ceiling: each lockstep group's kernel-counted levels (its deepest root's
    dependent block loads, summed over simulations) x the load latency; the probe latency interpolates
    between the measured footprints and walks per wave"""
    import numpy as np

    import bench

    S = 50
    pl = bench.search_plan(S, 8192)  # cooperative: 32-root workgroups, 256 of them = one round
    levels = np.full(256, 3 * S)
    levels[7] = 5 * S  # the slowest group: 5 levels per simulation
    f = bench.tree_latency_model(levels, S, pl, 8192, kernel_ms=1.0)
    assert f["roots_per_group"] == 32 and f["groups"] == 256 and f["rounds"] == 1
    assert abs(f["levels_per_sim"]["max_group"] - 5.0) < 1e-12
    assert abs(f["floor_ms"] - 5 * S * bench.TREE_LOAD_NS * 1e-6) < 1e-12
    assert abs(f["model_ms"] - 5 * S * f["model_load_ns"] * 1e-6) < 1e-12 and f["frac"] == f["model_ms"]
    # 8 walks per wave (the 32-root tile's waves), 8,192 x 51 x 128 B = 51 MB: between the probe's points
    assert bench.TREE_PROBE_NS[(16, 8)] < f["model_load_ns"] < bench.TREE_PROBE_NS[(128, 8)]
    pw = bench.search_plan(S, 262144)  # wave kernel: 32-root waves, 8,192 waves = 4 rounds of 2,048 slots
    f = bench.tree_latency_model(np.full(8192, 2 * S), S, pw, 262144)
    assert f["roots_per_group"] == 32 and f["rounds"] == 4
    assert abs(f["model_ms"] - 4 * 2 * S * bench.TREE_PROBE_NS[(1344, 32)] * 1e-6) < 1e-9
    assert bench.probe_latency_ns(448, 32) == bench.TREE_PROBE_NS[(448, 32)]


def test_traffic_summary_keeps_the_bench_instantiation(tmp_path):
    """tools/traffic.py: a profiled bench command that also launched another instantiation of the
    same kernel (the minmax_in leg's MMIN = true) summarises the bench's own instantiation as
    'fused' and lists the other under 'other', kept out of the PMC figures"""
    import csv

    import traffic

    bench_k = "mzh_search_kernel<32, false, true, true, false>"
    other_k = "mzh_search_kernel<32, false, true, true, true>"
    tree_k = "mzh_search_kernel<32, true, false, true, false>"
    full = lambda k: f"void {k}(MzhNet, MzhSearchParams)"  # noqa: E731
    d = tmp_path / "prof_t_trace" / "run"
    d.mkdir(parents=True)
    with open(d / "1_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "AverageNs"])
        w.writerow([full(bench_k), 12, 1300000.0])
        w.writerow([full(other_k), 6, 1250000.0])  # listed after the bench's: must not overwrite it
        w.writerow([full(tree_k), 12, 250000.0])
    d = tmp_path / "prof_t_fetch" / "run"
    d.mkdir(parents=True)
    with open(d / "1_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Dispatch_Id", "Counter_Value"])
        for disp, k, v in ((1, bench_k, 100.0), (2, bench_k, 100.0), (3, other_k, 999.0), (4, tree_k, 10.0)):
            for xcd in range(2):  # per-XCD rows of one dispatch are summed
                w.writerow([full(k), "FETCH_SIZE", disp, v / 2])
    out = traffic.summarise(str(tmp_path), "t", {"fused": bench_k, "tree": tree_k})
    assert out["fused"]["kernel"] == full(bench_k) and out["fused"]["avg_ns"] == 1300000.0
    assert out["fused"]["FETCH_SIZE"] == 100.0 and out["fused"]["hbm_read_bytes_corrected"] == 100.0 * 1024 * 2
    assert out["tree"]["kernel"] == full(tree_k) and out["tree"]["FETCH_SIZE"] == 10.0
    assert list(out["other"]) == [full(other_k)]


def _bench_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_n_without_launcher_starts_n_ranks():
    """`python bench.py --gpus 2` with no launcher must not print a 1-GPU line: it starts
    torch.distributed.run with 2 ranks itself (gloo, --dry-run: the rank plumbing without a GPU)"""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--dry-run"], capture_output=True, text=True, timeout=300, env=_bench_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dist"]["world_size"] == 2 and rec["dist"]["backend"] == "gloo"
    assert sorted(rec["dist"]["ranks"]) == [0, 1] and sum(rec["dist"]["roots_per_rank"]) == 65536


def test_gpus_mismatch_with_launcher_world_fails():
    """a launcher's WORLD_SIZE that differs from --gpus is an error, never a mislabelled line"""
    import subprocess

    env = _bench_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_empty_shard_is_rejected():
    """more ranks than roots: a clear error, not a crash on an empty launch"""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--roots-per-gpu", "0", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=_bench_env(), cwd=ROOT)
    assert r.returncode != 0 and "non-empty shard" in (r.stderr + r.stdout)


def test_launch_stats_and_abba_summary():
    """the line's kernel time is the median of the timed launches (one drifted launch cannot move frac);
    the caller-bounds leg is timed A B B A against plain launches of the same window"""
    import bench

    st = bench.launch_stats([6.2, 6.21, 6.4, 6.19, 6.2])
    assert st["n"] == 5 and st["min"] == 6.19 and st["max"] == 6.4 and st["median"] == 6.2
    assert abs(st["mean"] - 6.24) < 1e-12
    order = bench.abba_order(4)
    assert order == [0, 1, 1, 0] * 4 and order.count(0) == order.count(1) == 8
    # each leg follows each leg equally often: the predecessor mix is the same for A and B
    follows = {(a, b): 0 for a in (0, 1) for b in (0, 1)}
    for prev, cur in zip(order, order[1:]):
        follows[(prev, cur)] += 1
    assert follows[(0, 1)] == follows[(1, 0)]
    ab = bench.ab_summary([6.4, 6.2, 6.2, 6.3], [6.2, 6.2, 6.1, 6.3])
    assert ab["a"]["median"] == 6.25 and ab["b"]["median"] == 6.2
    assert abs(ab["ratio_median"] - 6.2 / 6.25) < 1e-12


def test_distinct_devices():
    """a multi-GPU record proves N physical devices by UUID (or PCI location) per host, not by world size"""
    import bench

    same = [{"host": "h", "uuid": "GPU-1", "device_index": 0}] * 2
    assert bench.distinct_devices(same) == 1
    eight = [{"host": "h", "uuid": f"GPU-{k}", "device_index": k} for k in range(8)]
    assert bench.distinct_devices(eight) == 8
    pci = [{"host": "h", "pci_bus_id": str(b), "pci_device_id": "0", "pci_domain_id": "0"} for b in (3, 3, 4)]
    assert bench.distinct_devices(pci) == 2
    assert bench.distinct_devices([{"host": "a", "device_index": 0}, {"host": "b", "device_index": 0}]) == 2


def test_gpus_8_driver_form_dry_run():
    """the exact N = 8 driver form (bench.py --gpus 8, self-launched) rehearsed on gloo without a GPU:
    8 ranks, every rank's LOCAL_RANK distinct, 8,192 roots each (configs[2] over 8 GPUs)"""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dist-backend", "gloo",
                        "--dry-run"], capture_output=True, text=True, timeout=600, env=_bench_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["dist"]["world_size"] == 8
    assert sorted(rec["dist"]["ranks"]) == list(range(8))
    assert rec["dist"]["roots_per_rank"] == [8192] * 8
    assert sorted(d["local_rank"] for d in rec["dist"]["devices"]) == list(range(8))
    assert [d["rank"] for d in rec["dist"]["devices"]] == list(range(8))
