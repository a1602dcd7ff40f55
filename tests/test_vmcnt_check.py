"""The load-completion checker run by build.py on the hand-pipelined device listings
(custereomatching_amd/vmcnt_check.py): no instruction may touch a VGPR whose load is still in flight.

Round 5 found the bug class it guards against: the compiler joined the backward sweep's prologue to its
loop with register copies of asm-load destinations before their `s_waitcnt`, so for k = 2..4 the first
call of a process (cold caches: late loads) copied what the previous wave had left in those registers.
Each rule is pinned on a synthetic listing; the shipped backward listing is checked in
tests/test_hazard_check.py (one compile for both checkers).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "custereomatching_amd"))
import vmcnt_check as vc  # noqa: E402

ASM = ";;#ASMSTART\n{}\n;;#ASMEND\n"
LD = "\tbuffer_load_dword v{}, v2, s[36:39], s26 offen"


def run(body, tmp_path):
    p = tmp_path / "k.s"
    p.write_text("_Zk:\n" + body + "\ts_endpgm\n.Lfunc_end0:\n")
    lines = p.read_text().split("\n")
    hits = []
    for _, (a, b) in vc.kernels(lines, []).items():
        hits += vc.check_kernel(lines, a, b)
    return sorted({(r[1], cons.op) for r, _, cons in hits})


def test_copy_before_the_wait_is_a_hit(tmp_path):
    body = ASM.format(LD.format(10)) + "\tv_mov_b32_e32 v20, v10\n\ts_waitcnt vmcnt(0)\n"
    assert run(body, tmp_path) == [(10, "v_mov_b32_e32")]
    body = ASM.format(LD.format(10)) + ASM.format("\ts_waitcnt vmcnt(0)") + "\tv_mov_b32_e32 v20, v10\n"
    assert run(body, tmp_path) == []


def test_reuse_as_temporary_is_a_hit(tmp_path):
    # the compiler may take a dead asm-load destination as scratch; the late load then overwrites it
    body = ASM.format(LD.format(10)) + "\tv_add_u32_e32 v10, v1, v2\n"
    assert run(body, tmp_path) == [(10, "v_add_u32_e32")]


def test_vmcnt_counts_younger_operations(tmp_path):
    # vmcnt(N) retires every operation with at least N younger ones (loads and stores alike)
    body = ASM.format(LD.format(10) + "\n" + LD.format(11)) + "\tbuffer_store_dword v3, v4, s[8:11], 0 offen\n"
    assert run(body + ASM.format("\ts_waitcnt vmcnt(1)") + "\tv_mov_b32_e32 v20, v11\n", tmp_path) == []
    assert run(body + ASM.format("\ts_waitcnt vmcnt(2)") + "\tv_mov_b32_e32 v20, v11\n", tmp_path) == [
        (11, "v_mov_b32_e32")]


def test_loop_back_edge_is_followed(tmp_path):
    # the load at the end of the body, the read at the head, the wait only on the exit path
    body = (".LBB0_1:\n\tv_mov_b32_e32 v20, v10\n" + ASM.format(LD.format(10)) +
            "\ts_cbranch_scc1 .LBB0_1\n\ts_waitcnt vmcnt(0)\n")
    assert run(body, tmp_path) == [(10, "v_mov_b32_e32")]


def test_wait_selected_by_a_lane_mask_flag(tmp_path):
    # the compiler's two-wait selection: a flag pair set to -1 / 0 and two vcc branches; a
    # path-insensitive analysis would see a path through neither wait
    body = (ASM.format(LD.format(10)) +
            "\tv_cmp_lt_i32_e32 vcc, s1, v1\n\ts_mov_b64 s[8:9], -1\n\ts_cbranch_vccz .LBB0_2\n" +
            ASM.format("\ts_waitcnt vmcnt(0)") + "\ts_mov_b64 s[8:9], 0\n"
            ".LBB0_2:\n\ts_andn2_b64 vcc, exec, s[8:9]\n\ts_cbranch_vccnz .LBB0_3\n" +
            ASM.format("\ts_waitcnt vmcnt(0)") + ".LBB0_3:\n\tv_mov_b32_e32 v20, v10\n")
    assert run(body, tmp_path) == []


def test_load_over_a_load_in_flight_is_allowed(tmp_path):
    # loads return in issue order: the later one wins; its address operand is still checked
    body = ASM.format(LD.format(10) + "\n" + LD.format(10)) + ASM.format("\ts_waitcnt vmcnt(0)")
    assert run(body, tmp_path) == []
    body = ASM.format(LD.format(2) + "\n" + LD.format(10)) + ASM.format("\ts_waitcnt vmcnt(0)")
    assert run(body, tmp_path) == [(2, "buffer_load_dword")]


def test_undefined_high_addend_of_a_32_bit_mad(tmp_path):
    body = ASM.format(LD.format(11)) + "\tv_mad_u64_u32 v[4:5], s[6:7], s18, 40, v[10:11]\n"
    assert run(body, tmp_path) == []
    body = ASM.format(LD.format(10)) + "\tv_mad_u64_u32 v[4:5], s[6:7], s18, 40, v[10:11]\n"
    assert run(body, tmp_path) == [(10, "v_mad_u64_u32")]
