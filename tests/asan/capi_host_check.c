/* Host-side AddressSanitizer check of the C ABI (SURVEY.md s5 "Race detection / sanitizers").
 *
 * Built by __graft_entry__.build_asan() against libadmm_deconv_asan.so -- the same library sources with
 * every host function instrumented (-Xarch_host -fsanitize=address; device code is not instrumented,
 * GPU sanitizers are not available on this pool).  Runs on a machine WITHOUT a GPU: it drives every
 * host-only path of the ABI -- workspace sizing over a sweep of shapes (the layout arithmetic the solve
 * carves its workspace with), argument validation of every entry point before any device work, the
 * options and profiler tables, and the thread-local error strings -- and exits 0 if every call returned
 * what the header promises.  ASan aborts (non-zero exit, report on stderr) on any out-of-bounds access,
 * use-after-free or leak in that host code.  tests/test_asan.py runs it. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "admm_deconv.h"
#include "admm_metrics.h"

static int failures = 0;
#define CHECK(cond)                                                             \
    do {                                                                        \
        if (!(cond)) {                                                          \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
            ++failures;                                                         \
        }                                                                       \
    } while (0)

static void sizes(void) {
    static const int shapes[][2] = {{2, 2},     {3, 5},     {64, 64},   {96, 96},   {250, 250}, {256, 256},
                                    {480, 640}, {512, 512}, {37, 29},   {1024, 16}, {2048, 2048}, {4096, 2}};
    for (size_t i = 0; i < sizeof(shapes) / sizeof(shapes[0]); ++i) {
        for (int iso = 0; iso < 2; ++iso) {
            for (int k = 0; k < 3; ++k) {
                const int M = shapes[i][0], N = shapes[i][1];
                const int kh = k == 0 ? 0 : (k == 1 ? 1 : (M < 15 ? M : 15));
                const int kw = k == 0 ? 0 : (k == 1 ? 1 : (N < 10 ? N : 10));
                size_t fw = 0, bw = 0, bwh = 0;
                CHECK(admm_tvd_workspace_bytes(M, N, 3, 5, kh, kw, iso, &fw) == ADMM_OK);
                CHECK(fw > 0);
                CHECK(admm_tvd_backward_workspace_bytes(M, N, 3, 5, kh, kw, iso, 7, 0, &bw) == ADMM_OK);
                CHECK(admm_tvd_backward_workspace_bytes(M, N, 3, 5, kh, kw, iso, 7, kh > 0, &bwh) == ADMM_OK);
                CHECK(bw >= fw && bwh >= bw);
            }
        }
    }
    size_t mw = 0;
    CHECK(admm_metrics_workspace_bytes(256, 256, 3, 4, 11, 1, &mw) == 0 && mw > 0);
    /* the MALL-resident schedule (round 6): its workspace is n chunk workspaces, the query agrees with it */
    long long chunk = 0;
    int streams = 0;
    size_t w4 = 0, w1 = 0, one = 0;
    CHECK(admm_query_forward_schedule(512, 512, 0, 15, 768, &chunk, &streams) == ADMM_OK && chunk == 8 && streams == 4);
    CHECK(admm_tvd_workspace_bytes(512, 512, 3, 256, 15, 15, 0, &w4) == ADMM_OK);
    CHECK(admm_tvd_workspace_bytes(512, 512, 1, 8, 15, 15, 0, &one) == ADMM_OK);
    CHECK(admm_set_option(ADMM_OPT_MALL_STREAMS, 1) == ADMM_OK);
    CHECK(admm_tvd_workspace_bytes(512, 512, 3, 256, 15, 15, 0, &w1) == ADMM_OK);
    CHECK(admm_query_forward_schedule(512, 512, 0, 15, 768, &chunk, &streams) == ADMM_OK && chunk == 768 && streams == 1);
    CHECK(admm_set_option(ADMM_OPT_MALL_STREAMS, 4) == ADMM_OK);
    CHECK(w4 >= 4 * one && w4 < w1);
    CHECK(admm_query_forward_schedule(512, 512, 0, 15, 0, &chunk, &streams) == ADMM_E_INVALID);
}

static void validation(void) {
    char* fake = (char*)(1 << 20);   /* never dereferenced: every call below fails validation first */
    size_t ws = 0;
    CHECK(admm_tvd_workspace_bytes(8192, 64, 1, 1, 5, 5, 0, &ws) == ADMM_E_UNSUPPORTED);
    CHECK(strlen(admm_last_error()) > 0);
    CHECK(admm_tvd_workspace_bytes(64, 64, 0, 1, 5, 5, 0, &ws) == ADMM_E_INVALID);
    CHECK(admm_tvd_workspace_bytes(64, 64, 1, 1, 5, 5, 0, NULL) == ADMM_E_INVALID);
    CHECK(admm_tvd_forward_f32(NULL, (float*)fake, 64, 64, 1, 1, NULL, 0, 0, 0.1f, 1.0f, 0, 5, fake, 1u << 30,
                               NULL) == ADMM_E_INVALID);
    CHECK(admm_tvd_forward_f32((float*)fake, (float*)fake, 64, 64, 1, 1, NULL, 0, 0, NAN, 1.0f, 0, 5, fake,
                               1u << 30, NULL) == ADMM_E_INVALID);
    CHECK(admm_tvd_forward_f32((float*)fake, (float*)fake, 64, 64, 1, 1, NULL, 0, 0, 0.1f, 1.0f, 0, 5, fake, 16,
                               NULL) == ADMM_E_WORKSPACE);
    CHECK(strstr(admm_last_error(), "workspace") != NULL);
    CHECK(admm_tvd_backward_f32((float*)fake, NULL, (float*)fake, NULL, NULL, NULL, 64, 64, 1, 1, NULL, 0, 0, 0.1f,
                                1.0f, 0, 5, (float*)fake, fake, 1u << 30, NULL) == ADMM_E_INVALID);
    CHECK(admm_tvd_forward_dev_f32((float*)fake, (float*)fake, 64, 64, 1, 1, NULL, 0, 0, NULL, (float*)fake, 0, 5,
                                   fake, 1u << 30, NULL, NULL) == ADMM_E_INVALID);
    /* a replay on a workspace that holds no recording */
    CHECK(admm_tvd_backward_recorded_f32((float*)fake, (float*)fake, (float*)fake, NULL, NULL, NULL, 64, 64, 1, 1,
                                         NULL, 0, 0, 0.1f, 1.0f, 0, 5, (float*)fake, fake + 4096, 1u << 30, NULL,
                                         NULL) == ADMM_E_INVALID);
    /* round-6 entry points: validation before any device work */
    CHECK(admm_clamp_backward_f32(NULL, (float*)fake, (float*)fake, 16, 0.f, 1.f, NULL) == ADMM_E_INVALID);
    CHECK(admm_clamp_backward_f32(NULL, NULL, NULL, 0, 0.f, 1.f, NULL) == ADMM_OK);   /* n = 0: nothing to do */
    CHECK(admm_gmsd_backward_f32((float*)fake, (float*)fake, 64, 64, 1, 1, 0.0026f, 0.f, NULL, NULL, fake, 1u << 20,
                                 NULL) == ADMM_E_INVALID);
    CHECK(admm_gmsd_backward_f32((float*)fake, (float*)fake, 64, 64, 1, 1, 0.0026f, 0.f, NULL, (float*)fake, fake, 8,
                                 NULL) == ADMM_E_WORKSPACE);
    /* a long message must be truncated, not overflow the thread-local buffer */
    CHECK(admm_tvd_workspace_bytes(1 << 30, 1 << 30, 1, 1, 1 << 29, 1 << 29, 0, &ws) != ADMM_OK);
    CHECK(strlen(admm_last_error()) < 4096);
}

static void options_and_profiler(void) {
    int v = -1;
    for (int o = 0; o < ADMM_OPT_COUNT; ++o) CHECK(admm_get_option(o, &v) == ADMM_OK);
    CHECK(admm_get_option(ADMM_OPT_COUNT, &v) != ADMM_OK);
    CHECK(admm_get_option(-1, &v) != ADMM_OK);
    CHECK(admm_set_option(ADMM_OPT_COUNT + 5, 1) != ADMM_OK);
    CHECK(admm_set_option(ADMM_OPT_FUSED, 0) == ADMM_OK && admm_get_option(ADMM_OPT_FUSED, &v) == ADMM_OK && v == 0);
    CHECK(admm_set_option(ADMM_OPT_FUSED, 1) == ADMM_OK);
    double ms = -1.0;
    long long n = -1;
    CHECK(admm_profile_reset() == ADMM_OK);
    for (int c = 0; c < ADMM_K_COUNT; ++c) CHECK(admm_profile_get(c, &ms, &n) == ADMM_OK && n == 0);
    CHECK(admm_profile_get(ADMM_K_COUNT, &ms, &n) != ADMM_OK);
    CHECK(admm_profile_get(-3, &ms, &n) != ADMM_OK);
}

int main(void) {
    CHECK(admm_abi_version() == ADMM_ABI_VERSION);
    sizes();
    validation();
    options_and_profiler();
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("asan host check: ok\n");
    return 0;
}
