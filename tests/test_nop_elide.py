"""CPU tests of the build's DPP hazard-pad elision (tools/nop_elide.py) and of the
hazard check it relies on (tools/check_dpp_hazards.py): a marked pad pair is dropped
only where the DPP read after it stays outside its hazard window, unmarked pads and
unpaired marked pads are never touched, and the checker flags what the pads guard
against (a VALU write of the broadcast source less than two wait states before the
DPP read, a label inside the window)."""
import os
import sys

TOOLS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
sys.path.insert(0, TOOLS)

import check_dpp_hazards as chk  # noqa: E402
import nop_elide  # noqa: E402

HN = "\ts_nop 0 ; hnop"


def _func(body):
    return ["\t.text", "kern:", *body, "\ts_endpgm"]


def _check_lines(tmp_path, lines):
    p = tmp_path / "k.s"
    p.write_text("\n".join(lines) + "\n")
    return chk.check(str(p))[1]


def test_pair_dropped_when_the_source_is_old(tmp_path):
    body = ["\tv_mov_b64 v[4:5], 1.0",        # writes the DPP source ...
            "\tv_add_f64 v[8:9], v[10:11], v[12:13]",
            "\tv_add_f64 v[14:15], v[10:11], v[12:13]",   # ... three wait states back
            HN, HN,
            "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    out, dropped, kept = nop_elide.elide(_func(body), chk)
    assert (dropped, kept) == (1, 0)
    assert not any("hnop" in l for l in out)
    assert not _check_lines(tmp_path, out)


def test_pair_kept_when_the_source_was_just_written(tmp_path):
    body = ["\tv_add_f64 v[8:9], v[10:11], v[12:13]",
            "\tv_mov_b64 v[4:5], 1.0",        # the DPP source, written right before the pads
            HN, HN,
            "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    lines = _func(body)
    out, dropped, kept = nop_elide.elide(lines, chk)
    assert (dropped, kept) == (0, 1) and out == lines
    assert not _check_lines(tmp_path, out)
    # without the pads the checker flags the read
    bare = [l for l in lines if "hnop" not in l]
    assert _check_lines(tmp_path, bare)


def test_label_inside_the_window_keeps_the_pair(tmp_path):
    body = [".LBB0_1:", HN, HN,
            "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    out, dropped, kept = nop_elide.elide(_func(body), chk)
    assert (dropped, kept) == (0, 1)


def test_unmarked_and_unpaired_pads_untouched():
    body = ["\ts_nop 0", "\ts_nop 0",          # alignment / M0 pads: no marker
            "\tv_add_f64 v[8:9], v[10:11], v[12:13]",
            "\tv_add_f64 v[14:15], v[10:11], v[12:13]",
            "\tv_add_f64 v[16:17], v[10:11], v[12:13]",
            HN,                                  # a single marked pad: its removal would
            "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    lines = _func(body)                          # shift the block's 8-byte alignment
    out, dropped, kept = nop_elide.elide(lines, chk)
    assert out == lines and dropped == 0


def test_exec_write_window_is_five(tmp_path):
    body = ["\ts_nop 0", "\tv_cmpx_lt_f64_e32 vcc, v[8:9], v[10:11]",
            "\tv_add_f64 v[14:15], v[10:11], v[12:13]", HN, HN,
            "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    out, dropped, kept = nop_elide.elide(_func(body), chk)
    assert (dropped, kept) == (0, 1)  # an EXEC write three states back: the pair stays
    assert _check_lines(tmp_path, out)  # (and the checker still reports the short window)


def test_lane_swap_writes_both_operands(tmp_path):
    """v_permlane16/32_swap (the pipelined rerun's slice gathers) rewrite both operands:
    a DPP read of the second one right after the swap is inside its window."""
    for op in ("v_permlane16_swap_b32_e32", "v_permlane32_swap_b32_e32"):
        w, _ = chk.vgpr_writes(f"{op} v6, v4")
        assert w == {6, 4}
        body = [f"\t{op} v6, v4",
                "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
        assert _check_lines(tmp_path, _func(body))


# ---------------------------------------------------------------------------
# round 6: gfx950's other software-managed hazards (tools/check_dpp_hazards.py
# docstring): one known-bad sequence per rule that the checker must reject, and the
# same sequence with enough wait states that it must accept
# ---------------------------------------------------------------------------

RULES = {
    # rule: (producer, consumer, wait states the consumer needs)
    "trans": ("\tv_rcp_f64_e32 v[4:5], v[6:7]",
              "\tv_fma_f64 v[8:9], v[4:5], v[10:11], v[12:13]", 1),
    "vmemsgpr": ("\tv_readfirstlane_b32 s7, v3",
                 "\tbuffer_load_dwordx4 v1, s[20:23], s7 offen nt lds", 5),
    "vmemsgpr_desc": ("\tv_readlane_b32 s23, v255, 7",
                      "\tbuffer_load_dwordx4 v1, s[20:23], s4 offen nt lds", 5),
    "rwlane": ("\tv_cmp_gt_f64_e64 s[10:11], 0, v[50:51]",
               "\tv_readlane_b32 s0, v254, s10", 4),
    "divfmas": ("\tv_div_scale_f64 v[30:31], vcc, v[32:33], v[32:33], v[84:85]",
                "\tv_div_fmas_f64 v[30:31], v[30:31], v[192:193], v[196:197]", 4),
    "readlane": ("\tv_add_f64 v[8:9], v[10:11], v[12:13]",
                 "\tv_readfirstlane_b32 s3, v8", 1),
    "permlane": ("\tv_add_f64 v[8:9], v[10:11], v[12:13]",
                 "\tv_permlane32_swap_b32_e32 v8, v20", 2),
    "m0lds": ("\ts_mov_b32 m0, s5",
              "\tbuffer_load_dwordx4 v1, s[20:23], s4 offen lds", 1),
}


def _seq(prod, cons, nops):
    return _func([prod] + ["\ts_nop 0"] * nops + [cons])


def test_each_rule_rejects_its_short_window_and_accepts_the_full_one(tmp_path):
    for rule, (prod, cons, ws) in RULES.items():
        short = _check_lines(tmp_path, _seq(prod, cons, ws - 1))
        assert short, (rule, "short window not flagged")
        assert any(rule.split("_")[0] in why for _, _, why in short), (rule, short)
        assert not _check_lines(tmp_path, _seq(prod, cons, ws)), (rule, "full window flagged")


def test_trans_rule_spares_a_trans_consumer_and_other_registers(tmp_path):
    # a transcendental reading a transcendental's result is not the forwarding case
    ok1 = _func(["\tv_rcp_f64_e32 v[4:5], v[6:7]", "\tv_sqrt_f64_e32 v[8:9], v[4:5]"])
    ok2 = _func(["\tv_rcp_f64_e32 v[4:5], v[6:7]", "\tv_fma_f64 v[8:9], v[14:15], v[10:11], v[12:13]"])
    assert not _check_lines(tmp_path, ok1) and not _check_lines(tmp_path, ok2)


def test_vmem_window_follows_a_branch_into_the_label(tmp_path):
    # the VALU SGPR write sits on the branch path, not the fall-through path
    body = ["\ts_cbranch_scc1 .LBB0_9", "\ts_nop 7", "\ts_nop 7", ".LBB0_9:",
            "\tbuffer_load_dwordx4 v1, s[20:23], s7 offen nt lds"]
    lines = _func(["\tv_readfirstlane_b32 s7, v3"] + body)
    assert _check_lines(tmp_path, lines)
    # with the producer far enough back on both paths, nothing is flagged
    assert not _check_lines(tmp_path, _func(["\tv_readfirstlane_b32 s7, v3", "\ts_nop 4"] + body))


def test_pad_inside_a_new_rule_window_is_kept(tmp_path):
    """The elider refuses a removal that opens any modelled window: here the pair is
    all that separates a v_rcp_f64 result from its non-transcendental consumer."""
    body = ["\tv_rcp_f64_e32 v[4:5], v[6:7]", HN, HN,
            "\tv_fma_f64 v[8:9], v[4:5], v[10:11], v[12:13]"]
    lines = _func(body)
    out, dropped, kept = nop_elide.elide(lines, chk)
    assert (dropped, kept) == (0, 1) and out == lines


VM = "\ts_nop 2 ; vmnop"


def test_vmem_pad_dropped_when_safe_and_kept_after_a_readlane(tmp_path):
    dma = ["\ts_mov_b32 s9, m0", "\ts_mov_b32 m0, s5", "\ts_nop 0",
           "\tbuffer_load_dwordx4 v1, s[20:23], s7 offen nt lds", "\ts_mov_b32 m0, s9"]
    safe = _func(["\tv_readfirstlane_b32 s7, v3", "\ts_nop 4", VM] + dma)
    out, dropped, kept = nop_elide.elide(safe, chk)
    assert (dropped, kept) == (1, 0) and not any("vmnop" in l for l in out)
    assert not _check_lines(tmp_path, out)
    risky = _func(["\tv_readlane_b32 s23, v255, 7", VM] + dma)
    out, dropped, kept = nop_elide.elide(risky, chk)
    assert (dropped, kept) == (0, 1) and out == risky
    assert not _check_lines(tmp_path, out)
    assert _check_lines(tmp_path, [l for l in risky if "vmnop" not in l])


def test_pads_split_by_an_alignment_directive_are_not_a_pair():
    """a marked pad, a .p2align, then the next block's marked pad: removing
    them as a pair would leave the block's 8-byte instructions at 4 mod 8."""
    body = ["\tv_add_f64 v[8:9], v[10:11], v[12:13]",
            "\tv_add_f64 v[14:15], v[10:11], v[12:13]",
            "\tv_add_f64 v[16:17], v[10:11], v[12:13]",
            HN, "\t.p2align 3", HN,
            "\tv_fmac_f64_dpp v[0:1], v[4:5], v[2:3] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    lines = _func(body)
    out, dropped, kept = nop_elide.elide(lines, chk)
    assert out == lines and dropped == 0


def _split(between):
    return ["\t.text", "kern:", "\t;;#ASMSTART",
            "\tds_read_b64 v[10:11], v2 offset:0", "\tds_read_b64 v[12:13], v2 offset:8 ; hop_ldissue",
            "\t;;#ASMEND", *between, "\t;;#ASMSTART", "\ts_waitcnt lgkmcnt(0) ; hop_ldwait",
            "\t;;#ASMEND", "\tv_add_f64 v[20:21], v[10:11], v[12:13]", "\ts_endpgm"]


def test_split_asm_load_destinations_untouched_until_the_wait(tmp_path):
    """ADVICE r05 (lft_sweep_v2.hip sym_issue13 / sym_wait_average13): nothing between
    the marked load statement and its marked wait may copy, spill or overwrite a load
    destination."""
    ok = _split(["\tv_add_f64 v[30:31], v[32:33], v[34:35]"])
    assert not _check_lines(tmp_path, ok)
    for bad in ("\tv_mov_b64_e32 v[40:41], v[12:13]",            # a copy before the data lands
                "\tscratch_store_dwordx2 off, v[10:11], s33",    # a spill
                "\tv_mov_b32_e32 v11, 0"):                       # the register reused
        assert _check_lines(tmp_path, _split([bad])), bad
    # no wait before the function ends
    lines = _split([])
    lines = [l for l in lines if "hop_ldwait" not in l]
    assert _check_lines(tmp_path, lines)
