"""The wait-state checker that guards the inline asm without `s_nop` (custereomatching_amd/
hazard_check.py, run by build.py on the device listings of bwd_fused.hip and sweep_wave.hip).

Each rule is checked on a synthetic listing: flagged at too few wait states, silent at enough,
through a loop back-edge, and not at all when neither side is inline asm.  The last test runs
the checker on the device listing of the shipped backward source (hipcc cross-compiles here).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "custereomatching_amd"))
import hazard_check as hc  # noqa: E402


def run(text, tmp_path):
    p = tmp_path / "k.s"
    p.write_text(text)
    lines = p.read_text().split("\n")
    hits = []
    for name, (a, b) in hc.kernels(lines, []).items():
        hits += [h for h in hc.check_kernel(lines, a, b) if h[3].asm or h[4].asm]
    return [(h[0], h[2]) for h in hits]


def kernel(body):
    return "_Zk:\n" + body + "\ts_endpgm\n.Lfunc_end0:\n"


ASM = ";;#ASMSTART\n{}\n;;#ASMEND\n"


@pytest.mark.parametrize("pad,expect", [(0, [("R1", 0)]), (3, [("R1", 3)]), (4, [("R1", 4)]), (5, [])])
def test_valu_sgpr_then_vmem(tmp_path, pad, expect):
    body = "\tv_readfirstlane_b32 s26, v3\n" + ("\ts_nop {}\n".format(pad - 1) if pad else "")
    body += ASM.format("\tbuffer_load_dword v1, v2, s[36:39], s26 offen")
    assert run(kernel(body), tmp_path) == expect


def test_dpp_source_needs_two_states(tmp_path):
    body = "\tv_mov_b32_e32 v7, v1\n" + ASM.format("\tv_mov_b32_dpp v8, v7 row_newbcast:1 row_mask:0xf bank_mask:0xf")
    assert run(kernel(body), tmp_path) == [("R2", 0)]
    body = "\tv_mov_b32_e32 v7, v1\n\tv_mov_b32_e32 v9, v1\n\tv_mov_b32_e32 v10, v1\n"
    body += ASM.format("\tv_mov_b32_dpp v8, v7 row_newbcast:1 row_mask:0xf bank_mask:0xf")
    assert run(kernel(body), tmp_path) == []


def test_permlane_swap_and_lane_select(tmp_path):
    body = "\tv_add_f32_e32 v5, v1, v2\n" + ASM.format("\tv_permlane32_swap_b32 v4, v5")
    assert run(kernel(body), tmp_path) == [("R3", 0)]
    body = ASM.format("\tv_cmp_eq_u32_e64 s[4:5], v1, v2\n\tv_readlane_b32 s9, v1, s4")
    assert run(kernel(body), tmp_path) == [("R4", 0)]


def test_loop_back_edge_is_followed(tmp_path):
    # the producer sits at the END of the loop body, the asm consumer at its START
    body = (".LBB0_1:\n" + ASM.format("\tv_mov_b32_dpp v8, v7 row_newbcast:1 row_mask:0xf bank_mask:0xf")
            + "\ts_add_i32 s0, s0, 1\n\tv_mov_b32_e32 v7, v1\n\ts_cbranch_scc1 .LBB0_1\n")
    # v_mov, then s_cbranch (1 state) -> the DPP at the loop head
    assert run(kernel(body), tmp_path) == [("R2", 1)]


def test_compiler_only_pairs_are_not_reported(tmp_path):
    body = "\tv_mov_b32_e32 v7, v1\n\tv_mov_b32_dpp v8, v7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
    assert run(kernel(body), tmp_path) == []


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None and shutil.which("hipcc") is None,
                    reason="no hipcc")
def test_shipped_backward_listing_is_clean(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else "hipcc"
    src = os.path.join(ROOT, "custereomatching_amd", "csrc", "bwd_fused.hip")
    out = tmp_path / "bwd.s"
    r = subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-gpu-rdc",
                        "--cuda-device-only", "-S", src, "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert hc.main(["hazard_check.py", str(out)]) == 0
    import vmcnt_check  # the same listing: no register read with its load in flight (tests/test_vmcnt_check.py)
    assert vmcnt_check.main(["vmcnt_check.py", str(out)]) == 0


def test_build_rejects_scratch_use():
    from custereomatching_amd.build import scratch_lines
    ok = "k_a:\n; ScratchSize: 0\n; Occupancy: 3\nk_b:\n; ScratchSize: 0\n"
    bad = "k_a:\n; ScratchSize: 0\nk_b:\n; ScratchSize: 28\n"
    assert scratch_lines(ok) == []
    assert scratch_lines(bad) == ["; ScratchSize: 28"]
