"""Build libmzh.so in-tree for gfx950 with hipcc (no JIT cache, no setuptools).

    python -m muzero_hanoi_amd.build          # or muzero_hanoi_amd.build.build()

-ffp-contract=off is part of the numerics contract (no implicit FMA contraction in the fp64
tree arithmetic or the fp32 epilogues; see csrc/mzh_device.h).
"""
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
REPO = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libmzh.so")
OBJ = os.path.join(HERE, "_obj")
SOURCES = ["mzh_api.hip", "mzh_search.hip", "mzh_wave.hip", "mzh_one.hip", "mzh_env.hip", "mzh_train.hip",
           "mzh_replay.hip"]
# host-only sources, compiled by g++ like the NumPy C code they restate (no -march: no FMA; see
# csrc/mzh_rng.cpp)
HOST_SOURCES = ["mzh_rng.cpp"]
HOST_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MZH_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-Wall", "-Wno-unused-result", "-I", os.path.join(REPO, "include")]
# per-source additions.  mzh_search.hip (the cooperative kernels, one wave per SIMD at 256 arch VGPRs):
# MFMA accumulators in arch VGPRs instead of the heuristic's AGPRs, so no epilogue element needs a
# v_accvgpr_read (8,192 roots -1.7%, 4,096 -2.0%; the wave kernels, built without it, measured neutral;
# profiles/r05_vgpr_form_ab.json).  Register allocation only: the same instructions, bit-identical results.
# mzh_one.hip (the latency kernel, 134 weight registers per lane at two waves per SIMD): no SLP vectorisation --
# it packs the interleaved policy / value chains into v_pk_fma_f32, which needs each weight pair in adjacent
# registers and copies the rows it shares with the other chains (231 spilled VGPRs with it, none in the loop
# without it)
SOURCE_FLAGS = {"mzh_search.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"], "mzh_one.hip": ["-fno-slp-vectorize"]}


BUILD_ID_MARKER = b"MZH_BUILD_ID:"


def source_files():
    """every file the library is compiled from: csrc/*.hip, csrc/*.cpp, csrc/*.h and include/mzh.h"""
    fs = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h")))
    return [os.path.join(CSRC, f) for f in fs] + [os.path.join(REPO, "include", "mzh.h")]


def source_hash(flags=None):
    """build id: sha256 over the sources' names and bytes and the compiler flags (first 20 hex)"""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    # flags without the checkout's absolute path (the GPU box runs the same tree from another path)
    h.update(" ".join(FLAGS if flags is None else flags).replace(REPO, "<repo>").encode())
    h.update(" ".join(HOST_FLAGS).encode())
    for src in sorted(SOURCE_FLAGS):
        h.update(f"{src}:{' '.join(SOURCE_FLAGS[src])}".encode())
    return h.hexdigest()[:20]


def embedded_build_id(lib_path):
    """the build id compiled into a built library (read from the file, without loading it)"""
    try:
        with open(lib_path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_MARKER)
    return None if i < 0 else data[i + len(BUILD_ID_MARKER): i + len(BUILD_ID_MARKER) + 20].decode("ascii", "replace")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, force=False, diag=False, tag="", defines=()):
    """diag=True builds libmzh_diag.so with -DMZH_STAMPS (in-kernel phase stamps; never shipped).
    tag/defines: an A/B variant of the diagnostic build (libmzh_diag_<tag>.so with -D<defines>)."""
    sfx = ("_diag" if diag else "") + (f"_{tag}" if tag else "")
    obj_dir = OBJ + sfx
    lib_path = LIB.replace("libmzh.so", f"libmzh{sfx}.so")
    # a define list entry starting with '-' is a compiler flag (e.g. -fno-slp-vectorize), else -D<entry>
    flags = FLAGS + (["-DMZH_STAMPS"] if diag else []) + [d if d.startswith("-") else f"-D{d}" for d in defines]
    os.makedirs(obj_dir, exist_ok=True)
    # the objects of a variant directory are only reusable for the same flags: a stamp file records
    # them, and a change forces a rebuild (A/B builds of one tag with different -D lists)
    stamp = os.path.join(obj_dir, "flags.txt")
    want = " ".join(flags)
    if not os.path.exists(stamp) or open(stamp).read() != want:
        force = True
    bid = source_hash(flags)
    if embedded_build_id(lib_path) != bid:
        force = True  # sources or flags differ from what the library was built from (not only mtimes)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(REPO, "include", "mzh.h"))
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, src.replace(".hip", ".o"))
        if force or _stale(o, [s] + headers):
            jobs.append([HIPCC, *flags, *SOURCE_FLAGS.get(src, []), "-c", s, "-o", o])
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, src.replace(".cpp", ".host.o"))
        if force or _stale(o, [s] + headers):
            jobs.append(["g++", *HOST_FLAGS, "-I", os.path.join(REPO, "include"), "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        for err in ex.map(run, jobs):
            if verbose and err:
                print(err, file=sys.stderr)
    objs = [os.path.join(obj_dir, s.replace(".hip", ".o")) for s in SOURCES]
    objs += [os.path.join(obj_dir, s.replace(".cpp", ".host.o")) for s in HOST_SOURCES]
    if force or jobs or _stale(lib_path, objs):
        # provenance: the build id as a host-only object linked into the library (mzh_build_id())
        id_src = os.path.join(obj_dir, "mzh_build_id.cpp")
        with open(id_src, "w") as f:
            f.write(f'static const char kId[] = "{BUILD_ID_MARKER.decode()}{bid}";\n'
                    'extern "C" const char* mzh_build_id(void) { return kId + %d; }\n' % len(BUILD_ID_MARKER))
        id_obj = os.path.join(obj_dir, "mzh_build_id.o")
        run(["g++", "-O2", "-fPIC", "-c", id_src, "-o", id_obj])
        run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, id_obj, "-o", lib_path,
             "-Wl,-rpath,/opt/rocm/lib", "-lm"])
    with open(stamp, "w") as f:
        f.write(want)
    with open(lib_path + ".flags", "w") as f:  # what this .so was built with (A/B logs cite it)
        f.write(want + "\n")
    return lib_path


if __name__ == "__main__":
    # --variant tag=DEF1,DEF2 : diagnostic A/B build libmzh_diag_<tag>.so
    var = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--variant=")]
    fvar = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--fast-variant=")]
    if fvar:  # timing A/B build without stamps: libmzh_<tag>.so
        tag, defs = fvar[0].split("=", 1) if "=" in fvar[0] else (fvar[0], "")
        print(build(verbose=True, force="--force" in sys.argv, diag=False, tag=tag,
                    defines=[d for d in defs.split(",") if d]))
    elif var:
        tag, defs = var[0].split("=", 1) if "=" in var[0] else (var[0], "")
        print(build(verbose=True, force="--force" in sys.argv, diag=True, tag=tag,
                    defines=[d for d in defs.split(",") if d]))
    else:
        print(build(verbose=True, force="--force" in sys.argv, diag="--diag" in sys.argv))
