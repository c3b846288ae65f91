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

CORE_CPU = ["cpu/generator.cpp", "cpu/cpu_tree.cpp", "cpu/protocol.cpp"]
CORE_HIP = ["gpu/build_global.hip", "gpu/build_subtree.hip", "gpu/query.hip", "gpu/dist_ops.hip",
            "gpu/generator.hip"]
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
               "-lamdhip64", f"-L{ROCM / 'lib'}", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{libdir}",
               f"-Wl,-rpath,{ROCM / 'lib'}"]
    return cflags, ldflags


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hdr_mtime() -> float:
    m = 0.0
    for d in (CSRC / "include", CSRC / "gpu", CSRC / "cli"):
        for p in d.rglob("*"):
            if p.suffix in (".hpp", ".h"):
                m = max(m, p.stat().st_mtime)
    return m


def _stale(out: Path, srcs, hdr: float) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(s).stat().st_mtime > t for s in srcs) or hdr > t


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def _compile(src: str, flags, verbose, hdr) -> Path:
    s = CSRC / src
    o = OBJ / (src.replace("/", "__") + ".o")
    if _stale(o, [s], hdr):
        if s.suffix == ".hip":
            cmd = [ROCM / "bin" / "hipcc", f"--offload-arch={ARCH}", *COMMON, *flags, "-c", s, "-o", o]
        else:
            cmd = ["g++", *COMMON, "-pthread", *flags, "-c", s, "-o", o]
        _run(cmd, verbose)
    return o


def build(verbose: bool = False, with_ext: bool = True, with_cli: bool = True, jobs: int | None = None) -> dict:
    """Compile every HIP/C++ source for gfx950 and link the extension + executables."""
    OBJ.mkdir(parents=True, exist_ok=True)
    BIN.mkdir(parents=True, exist_ok=True)
    hdr = _hdr_mtime()
    jobs = jobs or min(8, os.cpu_count() or 4)
    tflags, tld = _torch_flags() if with_ext else ([], [])
    tasks = [(s, []) for s in CORE_CPU + CORE_HIP]
    if with_ext:
        tasks += [(s, tflags) for s in BIND]
    if with_cli:
        hipflags = [f"-I{ROCM / 'include'}", "-D__HIP_PLATFORM_AMD__=1"]
        tasks += [(s, []) for v in CLI_CPU.values() for s in v]
        tasks += [(s, hipflags) for v in CLI_GPU.values() for s in v if (CSRC / s).exists()]
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {src: ex.submit(_compile, src, fl, verbose, hdr) for src, fl in tasks}
        objs = {src: f.result() for src, f in futs.items()}
    core_cpu = [objs[s] for s in CORE_CPU]
    core = core_cpu + [objs[s] for s in CORE_HIP]
    out = {}
    if with_ext:
        so = PKG / f"_C{_ext_suffix()}"
        srcs = core + [objs[s] for s in BIND]
        if _stale(so, srcs, 0.0):
            _run(["g++", "-shared", "-o", so, *srcs, *tld, "-pthread"], verbose)
        out["extension"] = str(so)
    if with_cli:
        for name, srcs in CLI_CPU.items():
            exe = BIN / name
            o = [objs[s] for s in srcs]
            if _stale(exe, o + core_cpu, 0.0):
                _run(["g++", "-o", exe, *o, *core_cpu, "-pthread"], verbose)
            out[name] = str(exe)
        for name, srcs in CLI_GPU.items():
            if not all(s in objs for s in srcs):
                continue
            exe = BIN / name
            o = [objs[s] for s in srcs]
            extra = ["-lrccl"] if name == "kdtree_dist" else []
            if _stale(exe, o + core, 0.0):
                _run(["g++", "-o", exe, *o, *core, f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrocprofiler-sdk-roctx", *extra,
                      f"-Wl,-rpath,{ROCM / 'lib'}", "-pthread"], verbose)
            out[name] = str(exe)
    return out


def clean():
    shutil.rmtree(ROOT / "build", ignore_errors=True)
    for p in PKG.glob("_C*.so"):
        p.unlink()
    for name in list(CLI_CPU) + list(CLI_GPU):
        (BIN / name).unlink(missing_ok=True)


if __name__ == "__main__":
    if "--clean" in sys.argv:
        clean()
    print(build(verbose="-v" in sys.argv))
