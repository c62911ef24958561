"""CPU-side checks of the boundary: libmzh.so loads, exports every symbol include/mzh.h declares,
the ctypes struct mirrors the C struct, and host logic behaves (no compute calls without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mzh.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(mzh_\w+)\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    from muzero_hanoi_amd import build

    build.build()
    from muzero_hanoi_amd import _lib

    return _lib


def test_library_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert len(syms) >= 15
    L = lib.lib()
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(lib.SIGNATURES), "ctypes signature table out of sync with include/mzh.h"
    assert L.mzh_abi_version() == lib.ABI_VERSION == 6


def _c_offsets(struct, fields, tmp_path):
    """offsetof of each field and sizeof of `struct` as the C compiler lays out include/mzh.h"""
    import shutil
    import subprocess

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / f"{struct}.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mzh.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof({struct}, {f}));\n' for f in fields)
                   + f'printf("%zu\\n", sizeof({struct})); return 0; }}\n')
    exe = tmp_path / struct
    subprocess.run([cc, "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    return [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]


def test_search_args_layout_matches_header(lib, tmp_path):
    """ctypes SearchArgs == struct mzh_search_args as the C compiler lays it out"""
    fields = [f[0] for f in lib.SearchArgs._fields_]
    want = [getattr(lib.SearchArgs, f).offset for f in fields] + [ctypes.sizeof(lib.SearchArgs)]
    assert _c_offsets("mzh_search_args", fields, tmp_path) == want
    hdr = open(HEADER).read()
    block = hdr[hdr.index("typedef struct mzh_search_args"):]
    block = block[:block.index("} mzh_search_args;")]
    n_ptr_fields = len(re.findall(r"^\s+(?:const\s+|struct\s+)?\w+\*\s+\w+;", block, re.M))
    assert n_ptr_fields == 19 == len(fields) - 7


def test_search_plan_layout_matches_header(lib, tmp_path):
    """ctypes SearchPlan == struct mzh_search_plan"""
    fields = [f[0] for f in lib.SearchPlan._fields_]
    want = [getattr(lib.SearchPlan, f).offset for f in fields] + [ctypes.sizeof(lib.SearchPlan)]
    assert _c_offsets("mzh_search_plan", fields, tmp_path) == want


def test_search_plan_query_names_the_instantiations(lib):
    """the host-only plan query (the code mzh_search launches from): kernel choice by batch size,
    cooperative tile, the one-hot-in-LDS and caller-bounds template arguments, forced kernels / tiles,
    the replay instantiation, capacity errors -- no device needed"""
    from muzero_hanoi_amd import engine

    P = lambda B, S=50, **kw: lib.search_plan(33, B, S, **kw)["kernel"]
    assert P(65536) == "mzh_wave_kernel<2, false, true>"
    assert P(53248) == "mzh_wave_kernel<2, false, true>"
    assert P(53247) == "mzh_wave_kernel<1, false, true>"
    assert P(8193) == "mzh_wave_kernel<1, false, true>"
    assert P(8192) == "mzh_search_kernel<32, false, true, true, false>"
    assert P(4097) == "mzh_search_kernel<32, false, true, true, false>"
    assert P(4096) == "mzh_search_kernel<16, false, true, true, false>"
    assert P(1025) == "mzh_search_kernel<16, false, true, true, false>"
    # the latency kernel: MLP searches of <= 512 roots (one root per workgroup, up to 256 workgroups;
    # the crossover with the cooperative kernel, profiles/r06_one_probe.json)
    # (the third argument: the latents in LDS, where they fit -- n_sims up to ~36)
    assert P(512) == P(1) == "mzh_search_one_kernel<true, false, false>"
    assert P(513) == "mzh_search_kernel<16, false, true, true, false>"
    assert P(1, minmax_in=True) == "mzh_search_one_kernel<true, true, false>"
    assert P(1, 25) == "mzh_search_one_kernel<true, false, true>"
    assert lib.search_plan(1, 1, 25)["kernel"] == "mzh_search_one_kernel<false, false, true>"
    pl = lib.search_plan(33, 500, 25)
    assert (pl["workgroups"], pl["roots_per_workgroup"], pl["threads_per_workgroup"]) == (256, 1, 512)
    assert lib.search_plan(33, 7, 25)["workgroups"] == 7
    assert P(1, replay=True) == "mzh_search_kernel<16, true, false, true, false>"  # no replay form
    assert P(1, 200) == "mzh_search_kernel<16, false, true, true, false>"  # its LDS does not fit: cooperative
    assert P(1, flags=engine.search_flags("coop")) == "mzh_search_kernel<16, false, true, true, false>"
    assert P(4096, flags=engine.search_flags("one")) == "mzh_search_one_kernel<true, false, false>"
    for bad in (dict(S=200), dict(replay=True), dict(flags=engine.search_flags("one", tile=16))):
        kw = dict(bad)
        S = kw.pop("S", 50)
        with pytest.raises((RuntimeError, ValueError), match="MZH_FLAG_KERNEL_ONE"):
            P(1, S, flags=kw.pop("flags", engine.search_flags("one")), **kw)
    # caller MinMaxStats bounds (every run_mcts / self-play search): one-hot table still in LDS
    assert P(4096, minmax_in=True) == "mzh_search_kernel<16, false, true, true, true>"
    assert P(8192, minmax_in=True) == "mzh_search_kernel<32, false, true, true, true>"
    assert P(65536, minmax_in=True) == "mzh_wave_kernel<2, false, true>"
    # replay (tree-only): one instantiation for both supports, never the LDS one-hot table
    assert P(8192, replay=True) == "mzh_search_kernel<32, true, false, true, false>"
    assert lib.search_plan(1, 8192, 50, replay=True)["kernel"] == "mzh_search_kernel<32, true, false, true, false>"
    assert lib.search_plan(1, 8192, 50)["kernel"] == "mzh_search_kernel<32, false, true, false, false>"
    assert lib.search_plan(1, 65536, 50, replay=True)["kernel"] == "mzh_wave_kernel<2, true, false>"
    # forced kernels / tiles
    assert P(8192, flags=engine.search_flags(tile=16)) == "mzh_search_kernel<16, false, true, true, false>"
    assert P(100, flags=engine.search_flags(tile=32)) == "mzh_search_kernel<32, false, true, true, false>"
    assert P(100, flags=engine.search_flags("wave")) == "mzh_wave_kernel<2, false, true>"
    assert P(100, flags=engine.search_flags("occ2")) == "mzh_search_occ2_kernel<true, false>"
    assert P(70000, flags=engine.search_flags("coop")) == "mzh_search_kernel<32, false, true, true, false>"
    assert P(70000, flags=engine.search_flags("wave16")) == "mzh_wave_kernel<1, false, true>"
    # deep trees: the 32-root tile's LDS path budget gives way to 16 roots, then to a capacity error
    big = lib.search_plan(33, 8192, 200)
    assert big["roots_per_workgroup"] in (16, 32) and big["smem_bytes"] <= 163840
    with pytest.raises(RuntimeError):
        lib.search_plan(33, 4096, 20000)
    pl = lib.search_plan(33, 8192, 50)
    assert (pl["wave"], pl["roots_per_workgroup"], pl["workgroups"], pl["threads_per_workgroup"]) == (0, 32, 256, 256)
    pl = lib.search_plan(33, 65536, 50)
    assert (pl["wave"], pl["roots_per_wave"], pl["workgroups"]) == (1, 32, 512)
    # the forced two-workgroups-per-CU kernel: served where its LDS fits twice per CU, an error where it
    # does not (no silent fallback), and replay searches name the cooperative replay kernel they run
    occ2 = engine.search_flags("occ2")
    assert P(8192, flags=occ2) == "mzh_search_occ2_kernel<true, false>"
    with pytest.raises(RuntimeError, match="MZH_FLAG_COOP_OCC2"):
        P(8192, 200, flags=occ2)
    assert P(8192, 200, flags=occ2, replay=True).startswith("mzh_search_kernel<")


def test_build_id_names_the_checked_out_sources(lib, tmp_path, monkeypatch):
    """provenance: the library carries the hash of the sources + flags it was built from, equal to
    the checked-out tree's; the hash moves with any source byte (the loader refuses a mismatch)"""
    import shutil

    from muzero_hanoi_amd import build

    want = build.source_hash()
    assert lib.build_id() == want == build.embedded_build_id(build.LIB)
    # a copy of the tree with one changed byte hashes differently
    csrc = tmp_path / "csrc"
    shutil.copytree(build.CSRC, csrc)
    with open(csrc / "mzh_tree.h", "a") as f:
        f.write("\n")
    monkeypatch.setattr(build, "CSRC", str(csrc))
    assert build.source_hash() != want
    # the GPU box runs the tree from another path: the checkout path is not part of the id
    monkeypatch.undo()
    assert build.source_hash([f.replace(build.REPO, "<repo>") for f in build.FLAGS]) == want
    # per-source flags (build.SOURCE_FLAGS: the cooperative kernels' register form) are part of the id too
    monkeypatch.setattr(build, "SOURCE_FLAGS", {k: [] for k in build.SOURCE_FLAGS})
    assert build.source_hash() != want


def test_train_args_layout_matches_header(lib, tmp_path):
    """ctypes TrainArgs == struct mzh_train_args as the C compiler lays it out"""
    fields = [f[0] for f in lib.TrainArgs._fields_]
    want = [getattr(lib.TrainArgs, f).offset for f in fields] + [ctypes.sizeof(lib.TrainArgs)]
    assert _c_offsets("mzh_train_args", fields, tmp_path) == want


def test_replay_args_layout_matches_header(lib, tmp_path):
    """ctypes ReplayArgs == struct mzh_replay_args as the C compiler lays it out"""
    fields = [f[0] for f in lib.ReplayArgs._fields_]
    want = [getattr(lib.ReplayArgs, f).offset for f in fields] + [ctypes.sizeof(lib.ReplayArgs)]
    assert _c_offsets("mzh_replay_args", fields, tmp_path) == want


def test_replay_argument_errors_are_loud(lib):
    """mzh_replay_sample / mzh_replay_set_priorities refuse bad shapes before touching a device"""
    L = lib.lib()
    a = lib.ReplayArgs()
    assert L.mzh_replay_sample(ctypes.byref(a), None) == lib.MZH_ERR_ARG
    a.n, a.m, a.d_state, a.U, a.A = 10, 4097, 9, 5, 6
    assert L.mzh_replay_sample(ctypes.byref(a), None) == lib.MZH_ERR_ARG and "m=4097" in lib.last_error()
    assert L.mzh_replay_set_priorities(None, 10, None, None, 4, None, None) == lib.MZH_ERR_ARG


def test_errors_without_device_are_loud(lib):
    if torch.cuda.is_available():
        pytest.skip("host without GPU only")
    L = lib.lib()
    h = ctypes.c_void_p()
    st = L.mzh_create(0, 4, 10, 10, 33, ctypes.byref(h))
    assert st == lib.MZH_ERR_HIP and not h.value
    assert "device" in lib.last_error()
    assert lib.device_count() == 0
    from muzero_hanoi_amd import engine

    with pytest.raises(RuntimeError):
        engine.Engine(4, 10, 10)


def test_argument_validation_without_device(lib):
    L = lib.lib()
    n = ctypes.c_size_t()
    assert L.mzh_weights_size(4, 33, ctypes.byref(n)) == 0
    assert n.value == 122824  # 122,824 params at N=4
    assert L.mzh_weights_size(3, 1, ctypes.byref(n)) == 0
    assert L.mzh_weights_size(0, 33, ctypes.byref(n)) == lib.MZH_ERR_ARG
    assert L.mzh_weights_size(4, 7, ctypes.byref(n)) == lib.MZH_ERR_ARG
    assert L.mzh_create(0, 0, 10, 10, 33, ctypes.byref(ctypes.c_void_p())) == lib.MZH_ERR_ARG
    assert L.mzh_env_step(0, 2, 10, 1, *([None] * 11)) == lib.MZH_ERR_ARG
    assert L.mzh_search(None, None, None) == lib.MZH_ERR_ARG
    with pytest.raises(ValueError):
        lib.check(lib.MZH_ERR_TEMPERATURE, "x")
    with pytest.raises(RuntimeError):
        lib.check(lib.MZH_ERR_HIP, "x")


def test_weight_flattening_matches_state_dict_order():
    from muzero_hanoi_amd import engine
    from muzero_hanoi_amd.networks import MuZeroNet
    from oracle import oracle as orc

    torch.manual_seed(0)
    net = MuZeroNet(12, 6, 0.002, "cpu", TD_return=True)
    flat = engine.flat_weights(net.state_dict())
    assert flat.size == 122824
    assert engine.WEIGHT_KEYS == orc.WEIGHT_KEYS
    # same seed -> the reference's initial weights (fixture from the reference itself)
    g = np.load(os.path.join(ROOT, "tests", "golden", "weights_N4_s0.npz"))
    for k in engine.WEIGHT_KEYS:
        assert np.array_equal(net.state_dict()[k].numpy(), g[k]), k


def test_dropin_torch_paths_match_reference_fixture():
    """MuZeroNet's torch methods (training/analysis path, not the HIP hot path) reproduce the
    reference's represent/prediction outputs on its own weights."""
    from muzero_hanoi_amd.networks import MuZeroNet

    torch.manual_seed(0)
    net = MuZeroNet(12, 6, 0.002, "cpu", TD_return=True)
    g = np.load(os.path.join(ROOT, "tests", "golden", "mlp_N4_s0.npz"))
    with torch.no_grad():
        h = net.represent(torch.tensor(g["x"]))
        pl, v = net.prediction(h)
    # batched torch GEMMs round differently from the reference's batch-1 calls: tolerances
    np.testing.assert_allclose(h.numpy(), g["ii_h"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(pl.numpy(), g["ii_policy_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(v.numpy()[:, 0], g["ii_value"], atol=2e-3, rtol=0)


def test_rng_predraw_consumes_like_reference():
    from muzero_hanoi_amd import rng

    np.random.seed(3)
    a = rng.predraw(5, deterministic=False, alpha=0.25)
    np.random.seed(3)
    manual = []
    for _ in range(5):
        d = np.random.dirichlet(np.ones(6, np.float32) * 0.25)
        t = np.random.choice(np.arange(6))
        u = np.random.random_sample()
        manual.append((d, t, u))
    assert np.array_equal(a[0], np.array([m[0] for m in manual]))
    assert np.array_equal(a[1], np.array([m[1] for m in manual]))
    assert np.array_equal(a[2], np.array([m[2] for m in manual]))
    n, t, u = rng.predraw(3, deterministic=True, alpha=0.25)
    assert n is None and u is None and t.shape == (3,)
