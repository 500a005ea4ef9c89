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
