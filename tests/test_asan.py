"""CPU: host-side AddressSanitizer run of the C ABI (SURVEY.md s5 "Race detection / sanitizers").

__graft_entry__.build() builds admm-deconv_amd/asan/: the library's host-logic translation units with
-Xarch_host -fsanitize=address (device code is not instrumented; GPU sanitizers are not available on
this pool) and tests/asan/capi_host_check.c, which drives every host-only path of the ABI without a GPU
(workspace layout over a shape sweep, argument validation of every entry point, options, profiler,
error strings).  ASan aborts the driver on any out-of-bounds access, use-after-free or leak."""
import os
import subprocess

ASAN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "admm-deconv_amd", "asan")


def test_asan_build_is_instrumented():
    out = subprocess.run(["nm", "-D", os.path.join(ASAN, "libadmm_deconv_asan.so")], capture_output=True,
                         text=True, check=True).stdout
    assert "__asan_report_load" in out


def test_capi_host_paths_under_asan():
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:detect_stack_use_after_return=1")
    r = subprocess.run([os.path.join(ASAN, "capi_host_check")], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan host check: ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "ERROR: LeakSanitizer" not in r.stderr
