"""Native build for gfx950 (no hipify, no JIT cache: everything lands in-tree).

Objects go to ``build/obj``; the PyTorch-ROCm extension is linked into
``parallel_kd_tree_amd/_C*.so`` and the CLI executables into ``bin/``. HIP sources are
compiled by ``hipcc --offload-arch=gfx950``; host C++ by g++. Everything uses
``-ffp-contract=off`` because squared distances must match the reference's separately
rounded multiply/add.

Usage: ``python -m parallel_kd_tree_amd._build [-v] [--clean]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "parallel_kd_tree_amd"
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
BIN = ROOT / "bin"
ARCH = os.environ.get("PKD_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

CORE_CPU = ["cpu/generator.cpp", "cpu/cpu_tree.cpp", "cpu/protocol.cpp", "cpu/tree_io.cpp", "cpu/global_plan.cpp"]
CORE_HIP = ["gpu/build_global.hip", "gpu/build_top.hip", "gpu/build_subtree.hip", "gpu/build_reference.hip", "gpu/query.hip",
            "gpu/dist_ops.hip", "gpu/generator.hip"]
HOST_HIP = ["cpu/global_builder.cpp", "cpu/tree_io_device.cpp"]  # host C++ on the HIP runtime (no device code)
BIND = ["bind/torch_bindings.cpp", "bind/dist_bindings.cpp"]
CLI_CPU = {"kdtree_sequential": ["cli/kdtree_sequential.cpp"]}
CLI_GPU = {"kdtree_gpu": ["cli/kdtree_gpu.cpp"], "kdtree_dist": ["cli/kdtree_dist.cpp"]}

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"-I{CSRC / 'include'}", f"-I{CSRC / 'gpu'}",
          "-Wall", "-Wno-unused-function"]


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [f"-I{sysconfig.get_paths()['include']}", f"-I{ROCM / 'include'}",
                                        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
                                        "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    libdir = Path(torch.__file__).parent / "lib"
    ldflags = [f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               "-lamdhip64", "-lrccl", f"-L{ROCM / 'lib'}", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{libdir}",
               f"-Wl,-rpath,{ROCM / 'lib'}"]
    return cflags, ldflags


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _digest(*parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def _hdr_digest() -> str:
    """Contents of every header a source may include."""
    parts = []
    for d in (CSRC / "include", CSRC / "gpu", CSRC / "cli"):
        for p in sorted(d.rglob("*")):
            if p.suffix in (".hpp", ".h"):
                parts += [p.relative_to(CSRC).as_posix(), p.read_bytes()]
    return _digest(*parts)


def _sig_path(out: Path) -> Path:
    return out.with_name(out.name + ".sig")


def _stale(out: Path, sig: str) -> bool:
    """An output is stale unless it exists and was built from exactly this signature
    (source and header contents, compiler, flags, offload arch) -- mtimes play no part, so a
    fresh checkout or a copied tree with up-to-date outputs rebuilds nothing."""
    sp = _sig_path(out)
    return not (out.exists() and sp.exists() and sp.read_text().strip() == sig)


def _mark(out: Path, sig: str) -> None:
    _sig_path(out).write_text(sig + "\n")


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def _obj_sig(src: str, flags, hdr: str) -> str:
    s = CSRC / src
    tool = f"hipcc --offload-arch={ARCH}" if s.suffix == ".hip" else "g++ -pthread"
    return _digest(src, s.read_bytes(), hdr, tool, *COMMON, *flags)


def _compile(src: str, flags, verbose, sig: str) -> Path:
    s = CSRC / src
    o = OBJ / (src.replace("/", "__") + ".o")
    if _stale(o, sig):
        if s.suffix == ".hip":
            cmd = [ROCM / "bin" / "hipcc", f"--offload-arch={ARCH}", *COMMON, *flags, "-c", s, "-o", o]
        else:
            cmd = ["g++", *COMMON, "-pthread", *flags, "-c", s, "-o", o]
        _run(cmd, verbose)
        _mark(o, sig)
    return o


LAST_BUILD = {"compiled": [], "seconds": 0.0}  # what the last build() in this process did


def build(verbose: bool = False, with_ext: bool = True, with_cli: bool = True, jobs: int | None = None) -> dict:
    """Compile every HIP/C++ source for gfx950 and link the extension + executables.

    Every output carries a signature (``<output>.sig``) of everything it was built from; an
    output whose signature matches is kept without looking at (or needing) its objects.
    Concurrent callers (the ranks of a multi-process run) serialise on a file lock: the first
    one builds, the others find every signature up to date."""
    import fcntl
    import time
    t0 = time.perf_counter()
    (ROOT / "build").mkdir(parents=True, exist_ok=True)
    with open(ROOT / "build" / ".build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            res, done = _build_locked(verbose, with_ext, with_cli, jobs)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    LAST_BUILD["compiled"] = done
    LAST_BUILD["seconds"] = time.perf_counter() - t0
    return res


def _build_locked(verbose, with_ext, with_cli, jobs):
    hdr = _hdr_digest()
    hipflags = [f"-I{ROCM / 'include'}", "-D__HIP_PLATFORM_AMD__=1"]
    tflags, tld = _torch_flags() if with_ext else ([], [])
    flags = {s: [] for s in CORE_CPU + CORE_HIP}
    flags.update({s: hipflags for s in HOST_HIP})
    if with_ext:
        flags.update({s: tflags for s in BIND})
    if with_cli:
        flags.update({s: [] for v in CLI_CPU.values() for s in v})
        flags.update({s: hipflags for v in CLI_GPU.values() for s in v if (CSRC / s).exists()})
    osig = {s: _obj_sig(s, fl, hdr) for s, fl in flags.items()}
    core_cpu, core = CORE_CPU, CORE_CPU + CORE_HIP + HOST_HIP
    # outputs: (path, object sources, link command tail)
    outs = {}
    if with_ext:
        outs["extension"] = (PKG / f"_C{_ext_suffix()}", core + BIND, [*tld, "-pthread"], ["-shared"])
    if with_cli:
        for name, srcs in CLI_CPU.items():
            outs[name] = (BIN / name, srcs + core_cpu, ["-pthread"], [])
        for name, srcs in CLI_GPU.items():
            if all(s in flags for s in srcs):
                extra = ["-lrccl"] if name == "kdtree_dist" else []
                outs[name] = (BIN / name, srcs + core, [f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrocprofiler-sdk-roctx",
                                                        *extra, f"-Wl,-rpath,{ROCM / 'lib'}", "-pthread"], [])
    lsig = {k: _digest(*(osig[s] for s in srcs), *tail, *pre) for k, (_, srcs, tail, pre) in outs.items()}
    todo = {k for k, (path, _, _, _) in outs.items() if _stale(path, lsig[k])}
    result = {k: str(path) for k, (path, _, _, _) in outs.items()}
    if not todo:
        return result, []
    OBJ.mkdir(parents=True, exist_ok=True)
    BIN.mkdir(parents=True, exist_ok=True)
    need = sorted({s for k in todo for s in outs[k][1]})
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {src: ex.submit(_compile, src, flags[src], verbose, osig[src]) for src in need}
        objs = {src: f.result() for src, f in futs.items()}
    for k in sorted(todo):
        path, srcs, tail, pre = outs[k]
        _run(["g++", *pre, "-o", path, *(objs[s] for s in srcs), *tail], verbose)
        _mark(path, lsig[k])
    return result, sorted(todo)


def clean():
    shutil.rmtree(ROOT / "build", ignore_errors=True)
    for p in list(PKG.glob("_C*.so")) + list(PKG.glob("_C*.so.sig")):
        p.unlink()
    for name in list(CLI_CPU) + list(CLI_GPU):
        (BIN / name).unlink(missing_ok=True)
        (BIN / f"{name}.sig").unlink(missing_ok=True)


if __name__ == "__main__":
    if "--clean" in sys.argv:
        clean()
    print(build(verbose="-v" in sys.argv))
