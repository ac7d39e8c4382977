"""Code-generation guards for the acting forward (CPU: hipcc cross-compiles gfx950 here).

k_qfc1 / k_qact2 keep their next chunks in registers while the current chunk's MFMAs run. Two
compiler behaviours silently undid that in round 4 ("The prefetch that did not
prefetch"): promote-alloca moved the staging arrays into LDS (every prefetch then waited
vmcnt(0)), and a prologue issuing its loads in another order than the loop made the s_waitcnt
pass wait for all but 2 loads in every iteration. These tests read the gfx950 assembly: no
private (scratch) segment, LDS exactly the declared tiles, and no wait inside k_qfc1's chunk loop
that drains the loads of the chunks ahead."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "maze-solving-agent-gymnasium_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")

pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")


@pytest.fixture(scope="module")
def qact_asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("asm") / "mz_qact.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "--cuda-device-only", "-S", "-o", str(out), "-I", CSRC,
                    os.path.join(CSRC, "mz_qact.hip")], check=True, capture_output=True)
    return out.read_text()


def kernel_meta(asm):
    meta, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"\s+\.amdhsa_kernel (\S+)", line)
        if m:
            cur = m.group(1)
            meta[cur] = {}
        m = re.match(r"\s+\.amdhsa_(group_segment_fixed_size|private_segment_fixed_size) (\d+)", line)
        if m and cur:
            meta[cur][m.group(1)] = int(m.group(2))
    return meta


def find(meta, part):
    names = [k for k in meta if part in k]
    assert names, part
    return names


def test_no_scratch_and_declared_lds_only(qact_asm):
    meta = kernel_meta(qact_asm)
    for part in ("k_qfc1", "k_qact2", "k_qconv"):
        for k in find(meta, part):
            assert meta[k]["private_segment_fixed_size"] == 0, k
    # k_qfc1: A[2 buffers][MZ_QFC1_CPB chunks][hi, lo][64 rows x 32 bf16]; k_qact2: A[2][hi, lo]
    # [64 x 32] + part[8][64][4] f32
    src = open(os.path.join(CSRC, "mz_qact.hip")).read()
    cpb = int(re.search(r"#define MZ_QFC1_CPB (\d+)", src).group(1))
    for k in find(meta, "k_qfc1"):
        assert meta[k]["group_segment_fixed_size"] == 2 * cpb * 2 * 64 * 32 * 2, k
    for k in find(meta, "k_qact2"):
        assert meta[k]["group_segment_fixed_size"] == 2 * 2 * 64 * 32 * 2 + 8 * 64 * 4 * 4, k


def test_qfc1_loop_keeps_loads_in_flight(qact_asm):
    """Inside k_qfc1's chunk loop every vmcnt wait leaves the next chunks' loads outstanding
    (10 per half-iteration: A(c+2) 2 + B(c+1) 8)."""
    start = qact_asm.index("k_qfc1E6MzQActiPKt:")
    body = qact_asm[start:qact_asm.index("s_endpgm", start)]
    waits, in_loop, hdr = [], False, None
    for ln in body.splitlines():
        m = re.match(r"(?:\.L(BB\d+_\d+)|; %bb\.\d+):", ln)
        if m:  # a block start: in the loop if it is the header or LLVM marks it "in Loop"
            if hdr is None and "Inner Loop Header" in ln:
                hdr = m.group(1)
            in_loop = hdr is not None and (m.group(1) == hdr or f"Header={hdr} " in ln + " ")
        if in_loop:
            w = re.search(r"vmcnt\((\d+)\)", ln)
            if w:
                waits.append(int(w.group(1)))
    assert waits, "no vmcnt waits found in the loop"
    assert min(waits) >= 8, waits
