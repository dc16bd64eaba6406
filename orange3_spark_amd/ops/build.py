"""In-tree build of the gfx950 kernel library.

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an object
and linked into ``ops/_lib/libo3s_kernels.so`` (C ABI, loaded by ``ops/_native.py``
through ctypes).  Host-only C++ runtime pieces (``csrc/*.cpp``) are compiled with the
same driver into ``ops/_lib/libo3s_host.so``.

No hipify, no CUDA sources, no torch JIT cache: the ``.so`` files live in the source
tree so they travel with the repository snapshot to the GPU box.

Usage: ``python -m orange3_spark_amd.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIBDIR = HERE / "_lib"
OBJDIR = LIBDIR / "obj"
ARCH = os.environ.get("O3S_OFFLOAD_ARCH", "gfx950")
KERNEL_LIB = LIBDIR / "libo3s_kernels.so"
HOST_LIB = LIBDIR / "libo3s_host.so"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build kernels)")


def _headers() -> list[Path]:
    return sorted(CSRC.glob("*.h"))


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + proc.stdout)


def _compile(src: Path, obj: Path, device: bool) -> Path:
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-c", str(src), "-o", str(obj),
           "-Wno-unused-result", "-I", str(CSRC)]
    if device:
        cmd[1:1] = [f"--offload-arch={ARCH}", "-ffp-contract=fast", "-munsafe-fp-atomics"]
    else:
        import sysconfig
        # host_strings.cpp reads str objects through the CPython headers; the symbols
        # resolve against the interpreter the library is loaded into (no libpython link)
        cmd[1:1] = ["-x", "c++", "-I", sysconfig.get_paths()["include"]]
    _run(cmd)
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> list[Path]:
    """Compile all sources that changed; return the produced library paths."""
    OBJDIR.mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    jobs = jobs or min(8, os.cpu_count() or 4)
    outs: list[Path] = []
    for lib, pattern, device in ((KERNEL_LIB, "*.hip", True), (HOST_LIB, "*.cpp", False)):
        srcs = sorted(CSRC.glob(pattern))
        if not srcs:
            continue
        todo, objs = [], []
        for s in srcs:
            o = OBJDIR / (s.stem + (".dev.o" if device else ".host.o"))
            objs.append(o)
            if force or _stale(o, [s, *hdrs]):
                todo.append((s, o))
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, s, o, device) for s, o in todo]
            for f in cf.as_completed(futs):
                o = f.result()
                if verbose:
                    print("compiled", o.name, flush=True)
        if force or _stale(lib, objs):
            cmd = [_hipcc(), "-shared", "-fPIC", "-o", str(lib), *map(str, objs)]
            if device:
                cmd.insert(1, f"--offload-arch={ARCH}")
            _run(cmd)
            if verbose:
                print("linked", lib, flush=True)
        outs.append(lib)
    return outs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    for p in build(force=a.force, jobs=a.jobs, verbose=True):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
