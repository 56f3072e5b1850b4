"""CPU: every `ccall` in julia/ADMMDeconvHIP.jl (the drop-in binding for /root/reference/src/ops/ops.jl:181,
never executed: Julia is absent) names an exported symbol and passes a type tuple that matches the C
prototype in include/admm_deconv.h argument for argument."""
import pytest

from admm_deconv import _lib
from julia_abi import JTYPES, c_prototypes, julia_ccalls

CALLS = julia_ccalls()


def test_shim_uses_the_device_scalar_entry_points():
    # λ / ρ stay on the device (the reference passes 1-element CuArrays, ops.jl:99,181)
    for name in ("admm_tvd_forward_dev_f32", "admm_tvd_forward_record_dev_f32", "admm_tvd_backward_recorded_dev_f32",
                 "admm_tvd_workspace_bytes", "admm_tvd_backward_workspace_bytes", "admm_last_error"):
        assert name in CALLS, name


@pytest.mark.parametrize("name", sorted(CALLS))
def test_ccall_types_match_prototype(name):
    protos = c_prototypes()
    assert name in protos and name in _lib.EXPORTS, name
    got = [JTYPES[t][0] for t in CALLS[name]]
    assert got == protos[name], f"{name}: julia {CALLS[name]} vs C {protos[name]}"


def test_shim_roots_what_it_passes_by_pointer():
    """Every ccall that passes device pointers sits inside a GC.@preserve block (the arrays must stay
    reachable while the call enqueues work on them)."""
    src = open(__import__("julia_abi").JL).read()
    for name in ("admm_tvd_forward_dev_f32", "admm_tvd_forward_record_dev_f32", "admm_tvd_backward_recorded_dev_f32"):
        i = src.index(f"ccall((:{name}")
        assert "GC.@preserve" in src[max(0, i - 200):i], name
