"""Host-side sanitizer build of the native extension: `_build --sanitize
address,undefined` compiles the launchers and torch bindings with ASan/UBSan (device code is
unchanged; GPU sanitizers are not used on this pool), and the library loads and registers its ops
under the sanitizer runtime."""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None or not Path("/opt/rocm/bin/hipcc").exists(),
                    reason="needs g++ and hipcc")
def test_host_sanitized_extension_builds_and_loads():
    from distributed_llm_alignment_amd import _build

    so = _build.build(sanitize="address,undefined")
    assert so.name == "_C_san.so" and so.exists()
    libs = []
    for name in ("libasan.so", "libubsan.so"):
        p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
        if not os.path.isabs(p):
            pytest.skip(f"{name} not found")
        libs.append(p)
    code = (
        "import torch\n"
        "from distributed_llm_alignment_amd.ops import _ext\n"
        "assert _ext.available(), _ext._STATE\n"
        "ns = torch.ops.dla\n"
        "for op in ('gg_fwd', 'attn_fwd', 'adamw_step', 'moe_dispatch'):\n"
        "    getattr(ns, op)\n"
        "print('SANITIZED_OK')\n")
    env = dict(os.environ, LD_PRELOAD=" ".join(libs), ASAN_OPTIONS="detect_leaks=0",
               DLA_EXT_PATH=str(so), PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300,
                       cwd="/tmp")
    assert "SANITIZED_OK" in r.stdout, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
