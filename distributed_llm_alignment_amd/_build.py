"""In-tree build of the gfx950 HIP extension (`distributed_llm_alignment_amd/_C.so`).

No hipify, no torch JIT cache: each `csrc/*.hip` is compiled by `hipcc --offload-arch=gfx950`
into an object (device code + plain C++ launchers), `csrc/bindings.cpp` (the TORCH_LIBRARY op
registry, host-only) by the host compiler against the installed torch headers, and everything is
linked into one shared object loaded with `torch.ops.load_library`. The `.so` lives next to this
file so it travels with the repository snapshot to the GPU box.

    python -m distributed_llm_alignment_amd._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
OUT_SO = PKG_DIR / "_C.so"
OBJ_DIR = PKG_DIR.parent / "build" / "dla_objs"
ARCH = os.environ.get("DLA_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_paths():
    import torch  # noqa: WPS433

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    lib = root / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hipcc() -> str:
    cand = ROCM / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


def _sources():
    hips = sorted(CSRC.glob("*.hip"))
    return hips, sorted(CSRC.glob("*.cpp"))


def _headers():
    return sorted(CSRC.glob("*.h"))


def _newer(src: Path, dst: Path, deps) -> bool:
    if not dst.exists():
        return True
    t = dst.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(map(str, cmd)) + "\n" + proc.stdout)
    return proc.stdout


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile every HIP kernel for gfx950 and link `_C.so`. Returns the .so path."""
    inc, lib, abi = _torch_paths()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hips, bindings = _sources()
    headers = _headers()
    jobs = jobs or min(8, os.cpu_count() or 4)
    hipcc = _hipcc()
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}"]
    tasks = []
    objs = []
    for src in hips:
        obj = OBJ_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            tasks.append([hipcc, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common,
                          "-c", str(src), "-o", str(obj)])
    cxx = shutil.which("g++") or shutil.which("c++") or "c++"
    py_inc = sysconfig.get_paths()["include"]
    for binding in bindings:  # host-only op registration (torch headers, g++)
        bobj = OBJ_DIR / (binding.stem + ".o")
        objs.append(bobj)
        if force or _newer(binding, bobj, headers):
            tasks.append([cxx, *common, f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
                          "-DUSE_ROCM=1", "-DHIPBLAS_V2", *[f"-I{p}" for p in inc],
                          f"-I{ROCM / 'include'}", f"-I{py_inc}", "-Wno-deprecated-declarations",
                          "-c", str(binding), "-o", str(bobj)])
    if tasks:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            for out in ex.map(_run, tasks):
                if verbose and out.strip():
                    print(out)
    if force or tasks or not OUT_SO.exists() or any(o.stat().st_mtime > OUT_SO.stat().st_mtime for o in objs):
        tmp = OUT_SO.with_suffix(".so.tmp")
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
              f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              f"-Wl,-rpath,{lib}"])
        os.replace(tmp, OUT_SO)
    return OUT_SO


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    so = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(f"built {so}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
