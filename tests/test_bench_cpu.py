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
    assert key == "hanoi4_s50_roots65536_wave"
    doc = json.load(open(os.path.join(ROOT, "profiles", "traffic_latest.json")))
    assert key in doc["entries"]
    ent = doc["entries"][key]
    assert ent["hbm_bytes_per_launch"] > 0 and ent["tree_hbm_bytes_per_launch"] > 0 and ent["build_id"]


def test_traffic_keys_of_every_config_and_shard():
    import bench

    assert bench.traffic_key(*bench.workload_shape(1)[:3]) == "hanoi4_s50_roots4096_coop"
    assert bench.traffic_key(*bench.workload_shape(3)[:3]) == "hanoi4_s200_roots16384_wave16"
    assert bench.traffic_key(*bench.workload_shape(2, world=8, rank=3)[:3]) == "hanoi4_s50_roots8192_coop"
    assert bench.traffic_key(*bench.workload_shape(4, world=8)[:3]) == "hanoi7_s100_roots32768_wave16"
    assert bench.traffic_key(*bench.workload_shape(2, roots_per_gpu=8192)[:3]) == "hanoi4_s50_roots8192_coop"


def test_traffic_is_reported_only_for_the_profiled_build(tmp_path):
    import bench

    from muzero_hanoi_amd import _lib, build

    build.build()
    key = "hanoi4_s50_roots65536_wave"
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
