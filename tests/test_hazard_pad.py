"""CPU unit tests of the build-time hazard pass (admm-deconv_amd/csrc/hazard_pad.py): a VALU write of a
data VGPR of a >64-bit VMEM store within 2 wait states is separated by s_nop, along the fallthrough, at
branches inside the window, and for the two-destination swap forms."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "admm-deconv_amd", "csrc"))
import hazard_pad  # noqa: E402

STORE = "\tbuffer_store_dwordx4 v[46:49], v189, s[24:27], s34 offen"


def pad(*lines):
    text, n = hazard_pad.pad_asm("\n".join(lines))
    return text.split("\n"), n


def test_valu_overwriting_store_data_is_padded():
    out, n = pad(STORE, "\tv_med3_f32 v48, v46, -s28, s28")
    assert n == 1 and out[1].strip() == "s_nop 1"


def test_unrelated_valu_is_not_padded():
    out, n = pad(STORE, "\tv_add_f32_e32 v50, v46, v47")
    assert n == 0


def test_narrow_store_is_not_a_hazard():
    out, n = pad("\tbuffer_store_dwordx2 v[46:47], v189, s[24:27], s34 offen", "\tv_mov_b32_e32 v46, 0")
    assert n == 0


def test_intervening_instructions_count_as_wait_states():
    _, n = pad(STORE, "\ts_mov_b32 s0, 1", "\tv_mov_b32_e32 v47, 0")
    assert n == 1                                   # one wait state spent, one missing
    out, n = pad(STORE, "\ts_nop 1", "\tv_mov_b32_e32 v47, 0")
    assert n == 0


def test_branch_inside_the_window_is_padded():
    out, n = pad(STORE, "\ts_cbranch_scc1 .LBB0_3", ".LBB0_3:", "\tv_mov_b32_e32 v48, 0")
    assert n == 1
    assert out[1].strip() == "s_nop 1" and out[2].strip().startswith("s_cbranch")
    out, n = pad(STORE, "\ts_branch .LBB0_7")
    assert n == 1 and out[1].strip() == "s_nop 1"


def test_branch_after_the_window_is_not_padded():
    _, n = pad(STORE, "\ts_nop 1", "\ts_branch .LBB0_7")
    assert n == 0


def test_swap_writes_both_operands():
    _, n = pad(STORE, "\tv_swap_b32 v10, v49")
    assert n == 1
    _, n = pad(STORE, "\tv_permlane32_swap_b32_e32 v12, v47")
    assert n == 1
    _, n = pad(STORE, "\tv_swap_b32 v10, v11")
    assert n == 0


@pytest.mark.parametrize("mn", ["global_store_dwordx4 v[0:1], v[46:49], off",
                                "global_store_dwordx3 v[0:1], v[46:48], off",
                                "scratch_store_dwordx4 off, v[46:49], s33 offset:16"])
def test_other_wide_store_forms(mn):
    _, n = pad("\t" + mn, "\tv_mov_b32_e32 v47, 0")
    assert n == 1


def test_scratch_sizes_reads_kernel_descriptors():
    """The build invariant check (__graft_entry__.TU_CHECKS) reads each kernel's scratch bytes from the
    .amdhsa_kernel descriptors of the device assembly."""
    import hazard_pad
    asm = """\t.amdhsa_kernel _Z3fooPf
\t\t.amdhsa_group_segment_fixed_size 0
\t\t.amdhsa_private_segment_fixed_size 0
\t.end_amdhsa_kernel
\t.amdhsa_kernel _Z3barPf
\t\t.amdhsa_private_segment_fixed_size 288
\t.end_amdhsa_kernel
"""
    assert hazard_pad.scratch_sizes(asm) == {"_Z3fooPf": 0, "_Z3barPf": 288}
