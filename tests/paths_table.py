"""The path every (shape, prox, PSF, call, record flags, options) combination must take -- the expected side of
admm_query_paths (admm_capi.hip plan_paths, the library's one decision table).  Shared by the CPU test
(tests/test_capi.py: the table against the query) and the GPU test (tests/test_gpu_paths.py: the kernels that
actually launch against the table).  mode: 0 forward, 1 record (flags = ADMM_REC_*), 2 combined backward."""

HBAR, MASKS = 1, 2
F, R, B = 0, 1, 2

# (id, M, N, iso, kh, mode, flags, want_hbar, want_rho, options, expected forward, expected sweep)
CASES = [
    ("c2-forward", 256, 256, False, 15, F, 0, False, False, {}, "fused", None),
    ("c2-forward-FUSED0", 256, 256, False, 15, F, 0, False, False, {"FUSED": 0}, "2pass", None),
    ("iso256-forward", 256, 256, True, 15, F, 0, False, False, {}, "fused_iso", None),
    ("iso256-forward-FUSED0", 256, 256, True, 15, F, 0, False, False, {"FUSED": 0}, "2pass_iso", None),
    ("c4-forward", 512, 512, False, 15, F, 0, False, False, {}, "2pass", None),
    ("iso512-forward", 512, 512, True, 0, F, 0, False, False, {}, "2pass_iso", None),
    ("250-forward", 250, 250, False, 15, F, 0, False, False, {}, "resident", None),
    ("240-forward", 240, 240, False, 15, F, 0, False, False, {}, "resident", None),
    ("96-forward", 96, 96, False, 0, F, 0, False, False, {}, "resident", None),
    ("250-forward-RESIDENT0", 250, 250, False, 15, F, 0, False, False, {"RESIDENT": 0}, "smooth", None),
    ("250-forward-SMOOTH0", 250, 250, False, 15, F, 0, False, False, {"SMOOTH": 0}, "runtime", None),
    ("250-iso-forward", 250, 250, True, 15, F, 0, False, False, {}, "resident_iso", None),
    ("250-iso-forward-RESIDENT0", 250, 250, True, 15, F, 0, False, False, {"RESIDENT": 0}, "smooth", None),
    ("480x640-forward", 640, 480, False, 15, F, 0, False, False, {}, "smooth", None),
    ("primes-forward", 37, 29, False, 5, F, 0, False, False, {}, "runtime", None),
    ("128-forward", 128, 128, False, 15, F, 0, False, False, {}, "resident", None),
    ("128-forward-RESIDENT0", 128, 128, False, 15, F, 0, False, False, {"RESIDENT": 0}, "2pass", None),
    ("96-iso-forward", 96, 96, True, 0, F, 0, False, False, {}, "resident_iso", None),
    ("32-iso-forward", 32, 32, True, 5, F, 0, False, False, {}, "resident_iso", None),
    ("128-forward-RESIDENT2", 128, 128, False, 15, F, 0, False, False, {"RESIDENT": 2}, "resident", None),
    ("demo32-record-RESIDENT2", 32, 32, False, 32, R, 0, False, False, {"RESIDENT": 2}, "resident", "sweep_2pass"),
    ("demo32-record-hbar-RESIDENT2", 32, 32, False, 32, R, HBAR, False, False, {"RESIDENT": 2}, "2pass", "sweep_2pass"),
    ("64-iso-RESIDENT2", 64, 64, True, 0, F, 0, False, False, {"RESIDENT": 2}, "resident_iso", None),
    ("250-iso-RESIDENT2", 250, 250, True, 15, F, 0, False, False, {"RESIDENT": 2}, "resident_iso", None),
    ("250-iso-record-RESIDENT2", 250, 250, True, 15, R, 0, False, False, {"RESIDENT": 2}, "resident_iso",
     "sweep_runtime_iso"),
    ("128-iso-backward-RESIDENT2", 128, 128, True, 0, B, 0, False, True, {"RESIDENT": 2}, "resident_iso",
     "sweep_2pass_iso"),
    ("128-iso-backward-hbar-RESIDENT2", 128, 128, True, 9, B, 0, True, True, {"RESIDENT": 2}, "2pass_iso",
     "sweep_2pass_iso"),
    # c5 layers: ADMMDeconvF2 (lambda trainable, rho fixed) records mask bits / the lane-native iso trajectory
    ("c5-record-masks", 256, 256, False, 0, R, MASKS, False, False, {}, "fused", "sweep_fused"),
    ("c5-record-full", 256, 256, False, 0, R, 0, False, False, {}, "fused", "sweep_fused"),
    ("c5-record-FUSED_ADJ0", 256, 256, False, 0, R, MASKS, False, False, {"FUSED_ADJ": 0}, "fused", "sweep_2pass"),
    ("c5iso-record-masks", 256, 256, True, 0, R, MASKS, False, False, {}, "fused_iso", "sweep_fused_iso"),
    ("c5iso-record-full", 256, 256, True, 0, R, 0, False, False, {}, "2pass_iso", "sweep_2pass_iso"),
    ("256-record-hbar", 256, 256, False, 15, R, HBAR, False, False, {}, "2pass", "sweep_2pass"),
    ("256-record-hbar-masks", 256, 256, False, 15, R, HBAR | MASKS, False, False, {}, "2pass", "sweep_2pass"),
    ("256-backward-norho", 256, 256, False, 15, B, 0, False, False, {}, "fused", "sweep_fused"),
    ("256-backward-rho", 256, 256, False, 15, B, 0, False, True, {}, "fused", "sweep_fused"),
    ("256-backward-hbar", 256, 256, False, 15, B, 0, True, True, {}, "2pass", "sweep_2pass"),
    ("iso256-backward-norho", 256, 256, True, 15, B, 0, False, False, {}, "fused_iso", "sweep_fused_iso"),
    ("iso256-backward-rho", 256, 256, True, 15, B, 0, False, True, {}, "2pass_iso", "sweep_2pass_iso"),
    ("c4-backward", 512, 512, False, 15, B, 0, True, True, {}, "2pass", "sweep_2pass"),
    ("250-record", 250, 250, False, 15, R, 0, False, False, {}, "resident", "sweep_runtime"),
    ("250-record-hbar", 250, 250, False, 15, R, HBAR, False, False, {}, "smooth", "sweep_runtime"),
    ("250-iso-backward", 250, 250, True, 15, B, 0, True, True, {}, "smooth", "sweep_runtime_iso"),
    ("primes-backward", 37, 29, False, 5, B, 0, True, True, {}, "runtime", "sweep_runtime"),
]

# The plane-count rule (ADMM_OPT_MIN_PLANES at its default, admm_capi.hip kMinPlanes): the one-workgroup-per-plane
# paths from the measured batch sizes where they beat the 2-pass kernels.  The table above queries with planes = 0
# (no rule), as its GPU test runs 2 planes with the rule off (conftest).
# (id, M, N, iso, kh, mode, flags, want_hbar, want_rho, planes, expected forward, expected sweep)
PLANE_CASES = [
    ("c2-95", 256, 256, False, 15, F, 0, False, False, 95, "2pass", None),
    ("c2-96", 256, 256, False, 15, F, 0, False, False, 96, "fused", None),
    ("c5-record-masks-64", 256, 256, False, 0, R, MASKS, False, False, 64, "2pass", "sweep_2pass"),
    ("c5-record-masks-96", 256, 256, False, 0, R, MASKS, False, False, 96, "fused", "sweep_fused"),
    ("256-backward-norho-8", 256, 256, False, 15, B, 0, False, False, 8, "2pass", "sweep_2pass"),
    ("iso256-forward-111", 256, 256, True, 15, F, 0, False, False, 111, "2pass_iso", None),
    ("iso256-forward-112", 256, 256, True, 15, F, 0, False, False, 112, "fused_iso", None),
    ("c5iso-record-masks-6", 256, 256, True, 0, R, MASKS, False, False, 6, "2pass_iso", "sweep_2pass_iso"),
    ("c5iso-record-masks-128", 256, 256, True, 0, R, MASKS, False, False, 128, "fused_iso", "sweep_fused_iso"),
    ("250-forward-128", 250, 250, False, 15, F, 0, False, False, 128, "smooth", None),
    ("250-forward-192", 250, 250, False, 15, F, 0, False, False, 192, "resident", None),
    ("250-record-64", 250, 250, False, 15, R, 0, False, False, 64, "smooth", "sweep_runtime"),
    ("128-forward-191", 128, 128, False, 15, F, 0, False, False, 191, "2pass", None),
    ("128-forward-192", 128, 128, False, 15, F, 0, False, False, 192, "resident", None),
    ("96-forward-6", 96, 96, False, 0, F, 0, False, False, 6, "resident", None),
    ("32-demo-forward-6", 32, 32, False, 32, F, 0, False, False, 6, "resident", None),
    ("96-iso-forward-255", 96, 96, True, 0, F, 0, False, False, 255, "smooth", None),
    ("96-iso-forward-256", 96, 96, True, 0, F, 0, False, False, 256, "resident_iso", None),
    ("250-iso-forward-255", 250, 250, True, 15, F, 0, False, False, 255, "smooth", None),
    ("250-iso-forward-256", 250, 250, True, 15, F, 0, False, False, 256, "resident_iso", None),
    ("32-iso-forward-6", 32, 32, True, 5, F, 0, False, False, 6, "2pass_iso", None),
]
