"""Build-time invariants of the kernels that name accumulator registers
literally: attn_fwd_v12 (csrc/flash_v12.hip), gemm_w4v and gemm_w5 (csrc/
gemm_w4v.hip, gemm_w5.hip; C^T in a[0:255]), CPU only.

The kernel names its accumulator registers literally in inline asm (O, Q, K
fragments in a[0:255]); hipcc does not know the Q fragments stay live between
the asm statements, so if it ever runs short of VGPRs it parks values in
those AGPRs (v_accvgpr_write/read of its own) and the Q fragments are
silently corrupted -- every output row of one 32-row block wrong.
$V12_DEFS adds -D switches (checking an A/B build before it goes to the GPU).  This
compiles the file the way build.py does and checks that no instruction
outside the asm statements touches an AGPR and that nothing spills.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "physics-llm-inference_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["flash_v12.hip", "gemm_w4v.hip", "gemm_w5.hip"])
def test_v12_no_compiler_agpr_use_or_spill(tmp_path, src):
    out = tmp_path / "k.s"
    flags = ["-fno-honor-nans"] if src == "flash_v12.hip" else []
    defs = os.environ.get("V12_DEFS", "").split() if src == "flash_v12.hip" else []
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950"] + flags + [
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-S", "--cuda-device-only",
           os.path.join(CSRC, src), "-o", str(out)] + defs
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    in_asm = False
    own = []
    for line in text.splitlines():
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        if not in_asm and re.search(r"\bv_accvgpr_(read|write)|\bscratch_(load|store)|buffer_(load|store).*off, s\[0:3\]",
                                    line):
            own.append(line.strip())
        # the LDS-DMA asm leaves M0 set between pieces (one write per four
        # pieces): nothing hipcc generates may read or write M0
        if not in_asm and re.search(r"\bm0\b", line.split(";")[0]):
            own.append(line.strip())
    assert not own, f"hipcc-generated AGPR/scratch/M0 accesses in {src}: {own[:8]}"
    sizes = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", text)]
    assert sizes and not any(sizes), f"{src}: a kernel uses scratch ({sizes})"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["flash_v13.hip", "flash_v13_d64.hip", "flash_pp64.hip"])
def test_v13_asm_only_kernels_build_clean(tmp_path, src):
    """attn_fwd_v13's bodies are one inline-asm statement each (tools/
    gen_flash_v13.py): the clobber list names no register hipcc reserves
    (no -Winline-asm warning: the program keeps off s32 / s100 / s101 and
    saves / restores m0 itself), no kernel has a stack frame or scratch, and
    no instruction hipcc generates outside the asm touches an AGPR, scratch,
    m0 or s32."""
    out = tmp_path / "k.s"
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-Winline-asm",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-S", "--cuda-device-only",
           os.path.join(CSRC, src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "inline asm clobber list contains reserved registers" not in r.stderr, r.stderr[-1500:]
    text = out.read_text()
    in_asm = False
    own = []
    for line in text.splitlines():
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        code = line.split(";")[0]
        if not in_asm and (re.search(r"\bv_accvgpr_(read|write)|\bscratch_(load|store)", code)
                           or re.search(r"\bm0\b|\bs32\b|\bs\[3[0-2]:", code)):
            own.append(line.strip())
    assert not own, f"hipcc-generated AGPR / scratch / m0 / s32 accesses in {src}: {own[:8]}"
    sizes = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", text)]
    assert sizes and not any(sizes), f"{src}: a kernel uses scratch ({sizes})"
