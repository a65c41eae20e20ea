"""Machine-code rules for the built gfx950 code object (CPU test: disassembles the device code
embedded in lib/libvr_amd.so, runs no kernel).

No FLAT memory instruction in any kernel.  Every buffer the kernels touch has a known address
space -- global (volume, TF, frame, tile lists) or LDS (staged TF) -- and a FLAT access whose
base and instruction offset straddle the LDS aperture is routed to the wrong aperture: the
round-4 non-pipelined march read its TF through one generic pointer chosen between LDS and
global, the compiler folded the +1 texel into a FLAT offset, and lookups of the low sentinel
(texel -1) faulted with MEMORY_APERTURE_VIOLATION (vr_kernels.hip tf_lookup).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "volumetric-renderer_amd", "lib", "libvr_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _disassembly(tmp_path):
    objdump = os.path.join(LLVM, "llvm-objdump")
    bundler = os.path.join(LLVM, "clang-offload-bundler")
    if not (os.path.exists(LIB) and os.path.exists(objdump) and os.path.exists(bundler)
            and shutil.which("objcopy")):
        pytest.skip("library or LLVM tools not present")
    fb = tmp_path / "fatbin.bin"
    co = tmp_path / "gfx950.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fb)],
                   check=True)
    subprocess.run([bundler, "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    out = subprocess.run([objdump, "-d", str(co)], check=True, capture_output=True, text=True)
    return out.stdout


def test_no_flat_memory_instructions(tmp_path):
    text = _disassembly(tmp_path)
    kernel = None
    hits = {}
    n_kernels = 0
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            kernel = m.group(1)
            n_kernels += 1
            continue
        if re.search(r"\bflat_(load|store|atomic)", line):
            hits.setdefault(kernel, 0)
            hits[kernel] += 1
    assert n_kernels > 50, "disassembly found too few kernels"
    assert not hits, hits
