"""In-tree build of the gfx950 HIP extension (`distributed_llm_alignment_amd/_C.so`).

No hipify, no torch JIT cache: each `csrc/*.hip` is compiled by `hipcc --offload-arch=gfx950`
into an object (device code + plain C++ launchers), `csrc/bindings.cpp` (the TORCH_LIBRARY op
registry, host-only) by the host compiler against the installed torch headers, and everything is
linked into one shared object loaded with `torch.ops.load_library`. The `.so` lives next to this
file so it travels with the repository snapshot to the GPU box.

    python -m distributed_llm_alignment_amd._build [--force] [-j N] [--sanitize address,undefined]

`--sanitize` (or DLA_SANITIZE=address,undefined) builds a host-sanitized variant into a separate
`_C_san.so` (select it with DLA_EXT_PATH=.../_C_san.so): the launchers, torch bindings and
argument checks run under ASan/UBSan, device code is unchanged (`-fsanitize=` goes after
`-Xarch_host` on every hipcc line; GPU-side sanitizers are not used on this pool). Use it for
host-code bugs in the C++ runtime; run with LD_PRELOAD of the matching libasan on a CPU box.
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
SAN_SO = PKG_DIR / "_C_san.so"
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


def _san_list(sanitize) -> list:
    if not sanitize:
        return []
    items = [x.strip() for x in str(sanitize).split(",") if x.strip()]
    bad = [x for x in items if x not in ("address", "undefined", "leak")]
    if bad:
        raise ValueError(f"unsupported host sanitizer(s) {bad}: address / undefined / leak")
    return items


def build(force: bool = False, jobs: int | None = None, verbose: bool = False,
          sanitize: str | None = None) -> Path:
    """Compile every HIP kernel for gfx950 and link `_C.so` (or the host-sanitized `_C_san.so`).
    Returns the .so path."""
    inc, lib, abi = _torch_paths()
    san = _san_list(sanitize if sanitize is not None else os.environ.get("DLA_SANITIZE_BUILD"))
    obj_dir = OBJ_DIR.parent / "dla_objs_san" if san else OBJ_DIR
    out_so = SAN_SO if san else OUT_SO
    obj_dir.mkdir(parents=True, exist_ok=True)
    hsan = [f"-Xarch_host -fsanitize={x}".split() for x in san]
    # vptr checks need the clang UBSan C++ runtime, which the g++-built bindings do not link; so
    # does clang's indirect-call type check (-fsanitize=function: __ubsan_handle_function_type_mismatch
    # is missing from g++'s libubsan, which is what the loader preloads)
    extra = ["-fno-omit-frame-pointer"] + (["-fno-sanitize=vptr"] if "undefined" in san else [])
    hextra = ["-fno-sanitize=function"] if "undefined" in san else []
    hsan = [a for pair in hsan for a in pair] + [a for x in extra + hextra for a in ("-Xarch_host", x)] if san else []
    gsan = [f"-fsanitize={x}" for x in san] + extra if san else []
    hips, bindings = _sources()
    headers = _headers()
    jobs = jobs or min(8, os.cpu_count() or 4)
    hipcc = _hipcc()
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}"]
    tasks = []
    objs = []
    for src in hips:
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            tasks.append([hipcc, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common, *hsan,
                          "-c", str(src), "-o", str(obj)])
    cxx = shutil.which("g++") or shutil.which("c++") or "c++"
    py_inc = sysconfig.get_paths()["include"]
    for binding in bindings:  # host-only op registration (torch headers, g++)
        bobj = obj_dir / (binding.stem + ".o")
        objs.append(bobj)
        if force or _newer(binding, bobj, headers):
            tasks.append([cxx, *common, *gsan, f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
                          "-DUSE_ROCM=1", "-DHIPBLAS_V2", *[f"-I{p}" for p in inc],
                          f"-I{ROCM / 'include'}", f"-I{py_inc}", "-Wno-deprecated-declarations",
                          "-c", str(binding), "-o", str(bobj)])
    if tasks:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            for out in ex.map(_run, tasks):
                if verbose and out.strip():
                    print(out)
    if force or tasks or not out_so.exists() or any(o.stat().st_mtime > out_so.stat().st_mtime for o in objs):
        tmp = out_so.with_suffix(".so.tmp")
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *hsan, "-o", str(tmp), *map(str, objs),
              f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lhipblaslt",
              f"-Wl,-rpath,{lib}"])
        os.replace(tmp, out_so)
    return out_so


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--sanitize", default=None, help="host sanitizers, e.g. address,undefined")
    a = ap.parse_args(argv)
    so = build(force=a.force, jobs=a.jobs, verbose=a.verbose, sanitize=a.sanitize)
    print(f"built {so}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
