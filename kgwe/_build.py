"""In-tree native build for kgwe (gfx950 only).

Produces, under ``kgwe/_lib/``:

* ``libkgwe_ops.so``    – hand-written HIP kernels for the training hot path
                           (RMSNorm, SwiGLU, RoPE, cross-entropy, AdamW,
                           flash attention) with a plain C ABI.
* ``libkgwe_probes.so`` – HBM / xGMI bandwidth probe kernels (topology
                           discovery), C ABI, no torch dependency.
* ``_kgwe_core*.so``    – the C++17 control-plane core (topology, scheduler,
                           partition planner, cost engine, metrics) as a
                           pybind11 module.

Everything is compiled with hipcc for ``--offload-arch=gfx950`` (hipcc
cross-compiles without a GPU) or g++ for the host-only core.  Objects are
cached by source mtime so a rebuild is incremental.

Usage: ``python -m kgwe._build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "kgwe" / "_lib"
OBJ = ROOT / "build" / "obj"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
    "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
    "-munsafe-fp-atomics",
    # No packed-FP32 VALU forms (v_pk_add/mul/fma_f32): hipcc -O3 otherwise
    # forms them from ordinary float code, and some of their forms have given
    # silently wrong results on this GPU pool.  (The host pass warns that it
    # does not know the feature; harmless.)
    "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
]
# Per-source extras.  flash_attn.hip: no SLP vectorisation — hipcc otherwise
# packs the softmax's adjacent f32 adds / multiplies into v_pk_*_f32, which
# costs more than two plain VALU ops when issued beside MFMAs
# (MI355X_MICROARCH.md); outputs are bit-identical, fwd / bwd +0.5-1 %
# (`tools/gpu.sh fa-variants`, variant "noslp").
HIP_FILE_FLAGS = {"flash_attn.hip": ["-fno-slp-vectorize"]}
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wextra",
             "-Wno-unused-parameter"]


def _sources(sub: str, exts=(".hip",)) -> list[Path]:
    d = ROOT / "native" / sub
    return sorted(p for p in d.iterdir() if p.suffix in exts)


def _headers(sub: str) -> list[Path]:
    d = ROOT / "native" / sub
    return sorted(p for p in d.iterdir() if p.suffix in (".h", ".hpp"))


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _compile(src: Path, compiler: str, flags: list[str], incs: list[Path],
             force: bool) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    obj = OBJ / (src.parent.name + "_" + src.name + ".o")
    deps = [src] + [h for inc in incs for h in inc.glob("*.h*")]
    if force or _stale(obj, deps):
        cmd = [compiler, *flags, *[f"-I{i}" for i in incs], "-c", str(src), "-o", str(obj)]
        _run(cmd)
    return obj


def _link(objs: list[Path], out: Path, linker: str, extra: list[str], force: bool) -> Path:
    LIB.mkdir(parents=True, exist_ok=True)
    if force or _stale(out, objs):
        _run([linker, "-shared", "-fPIC", *[str(o) for o in objs], "-o", str(out), *extra])
    return out


def build_ops(force: bool = False, jobs: int = 8) -> Path:
    srcs = _sources("ops")
    inc = [ROOT / "native" / "ops"]
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, HIPCC, HIP_FLAGS + HIP_FILE_FLAGS.get(s.name, []),
                                              inc, force), srcs))
    return _link(objs, LIB / "libkgwe_ops.so", HIPCC,
                 [f"--offload-arch={ARCH}", "-lamdhip64"], force)


def build_probes(force: bool = False, jobs: int = 8) -> Path:
    srcs = _sources("probes")
    inc = [ROOT / "native" / "probes"]
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, HIPCC, HIP_FLAGS, inc, force), srcs))
    return _link(objs, LIB / "libkgwe_probes.so", HIPCC,
                 [f"--offload-arch={ARCH}", "-lamdhip64", "-ldl"], force)


def build_core(force: bool = False, jobs: int = 8) -> Path | None:
    core_dir = ROOT / "native" / "core"
    srcs = sorted(core_dir.glob("*.cpp"))
    if not srcs:
        return None
    import pybind11  # noqa: PLC0415

    incs = [core_dir, Path(pybind11.get_include()), Path(sysconfig.get_paths()["include"]),
            Path("/opt/rocm/include")]
    cxx = os.environ.get("CXX", "g++")
    flags, link = list(CXX_FLAGS), ["-ldl", "-lpthread"]
    if os.environ.get("KGWE_CORE_SANITIZE") == "1":
        # Host-only ASan + UBSan build of the platform core (the role of the
        # reference's `go test -race`); load with LD_PRELOAD=libasan.so.
        san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
        flags += san
        link += san
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, cxx, flags, incs, force), srcs))
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return _link(objs, LIB / f"_kgwe_core{suffix}", cxx, link, force)


SANITIZERS = {
    "plain": [],
    "tsan": ["-fsanitize=thread"],
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
}


def build_native_tests(flavour: str = "plain", force: bool = False, jobs: int = 8) -> Path:
    """Standalone C++ test binary over the platform core (no pybind11, no
    Python): ``build/tests/core_tests_<flavour>``.  ``tsan`` / ``asan`` are
    the host-side race / memory-error builds."""
    core_dir = ROOT / "native" / "core"
    test_dir = ROOT / "native" / "tests"
    srcs = [s for s in sorted(core_dir.glob("*.cpp")) if s.name != "bindings.cpp"]
    srcs += sorted(test_dir.glob("*.cpp"))
    incs = [core_dir, Path("/opt/rocm/include")]
    cxx = os.environ.get("CXX", "g++")
    san = SANITIZERS[flavour]
    flags = ["-O1" if san else "-O2", "-g", "-std=c++17", "-Wall", "-Wextra",
             "-Wno-unused-parameter", "-fno-omit-frame-pointer", *san]
    global OBJ
    saved, OBJ = OBJ, ROOT / "build" / f"obj-tests-{flavour}"
    try:
        with cf.ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(lambda s: _compile(s, cxx, flags, incs, force), srcs))
    finally:
        OBJ = saved
    out = ROOT / "build" / "tests" / f"core_tests_{flavour}"
    out.parent.mkdir(parents=True, exist_ok=True)
    if force or _stale(out, objs):
        _run([cxx, *san, *[str(o) for o in objs], "-o", str(out), "-ldl", "-lpthread"])
    return out


def build_all(force: bool = False, jobs: int = 8) -> list[Path]:
    out = []
    with cf.ThreadPoolExecutor(3) as ex:
        futs = [ex.submit(build_ops, force, jobs), ex.submit(build_probes, force, jobs),
                ex.submit(build_core, force, jobs)]
        for f in futs:
            p = f.result()
            if p is not None:
                out.append(p)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--native-tests", choices=sorted(SANITIZERS), action="append",
                    help="also build the standalone C++ core test binary (flavour)")
    a = ap.parse_args(argv)
    for fl in a.native_tests or []:
        print(build_native_tests(fl, a.force, a.jobs).relative_to(ROOT))
    for p in build_all(a.force, a.jobs):
        print(p.relative_to(ROOT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
