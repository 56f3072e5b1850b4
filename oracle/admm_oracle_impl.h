/* CPU oracle body, instantiated for float and double by admm_oracle.c.
 * TEST INFRASTRUCTURE ONLY (see admm_oracle.c header).  Restates
 * /root/reference/src/ops/ops.jl:17-96 (tvd_fft_cpu) op for op:
 *   - Sigma, Lambda_x, Lambda_y by FFT of the zero-padded PSF / difference filters  (:22-36)
 *   - C = 1 / (|Sigma|^2 + rho (|Lx|^2 + |Ly|^2))                                    (:37)
 *   - per iteration: H^T(y) by SPATIAL circular correlation (re-evaluated every
 *     iteration exactly like the reference, :86), D^T(z-u) by the periodic 2x2 stencil,
 *     rfft2 -> xC -> irfft2, D(x), prox (ST or BT), dual update                       (:84-92)
 * Layout: y, x are float[B][P][N][M] (= Julia (M,N,P,B)); h is float[kw][kh].
 */
#ifndef R
#error "define R (real type) and SFX (suffix) before including"
#endif

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

typedef struct { R re, im; } FN(cpx_);
#define CPX FN(cpx_)

/* ---- FFT: radix-2 iterative for powers of two, naive DFT otherwise ------------------- */
typedef struct {
    int n, pow2;
    CPX *tw;     /* n/2 forward twiddles exp(-2 pi i k / n) (pow2) or n (dft) */
    int *rev;    /* bit reversal (pow2) */
} FN(plan_);
#define PLAN FN(plan_)

static void FN(plan_init)(PLAN *p, int n) {
    p->n = n;
    p->pow2 = (n & (n - 1)) == 0;
    int ntw = p->pow2 ? (n / 2 > 0 ? n / 2 : 1) : n;
    p->tw = (CPX *)malloc(sizeof(CPX) * ntw);
    for (int k = 0; k < ntw; ++k) {
        double a = -2.0 * M_PI * (double)k / (double)n;
        p->tw[k].re = (R)cos(a);
        p->tw[k].im = (R)sin(a);
    }
    p->rev = NULL;
    if (p->pow2) {
        int lg = 0;
        while ((1 << lg) < n) ++lg;
        p->rev = (int *)malloc(sizeof(int) * n);
        for (int i = 0; i < n; ++i) {
            int r = 0;
            for (int b = 0; b < lg; ++b) r |= ((i >> b) & 1) << (lg - 1 - b);
            p->rev[i] = r;
        }
    }
}

static void FN(plan_free)(PLAN *p) {
    free(p->tw);
    free(p->rev);
}

/* in-place complex FFT of a contiguous buffer; inv != 0 -> unnormalised inverse */
static void FN(fft)(const PLAN *p, CPX *a, CPX *scratch, int inv) {
    const int n = p->n;
    if (n == 1) return;
    if (p->pow2) {
        for (int i = 0; i < n; ++i) {
            int r = p->rev[i];
            if (r > i) { CPX t = a[i]; a[i] = a[r]; a[r] = t; }
        }
        for (int len = 2; len <= n; len <<= 1) {
            const int half = len >> 1, step = n / len;
            for (int s = 0; s < n; s += len) {
                for (int k = 0; k < half; ++k) {
                    CPX w = p->tw[k * step];
                    if (inv) w.im = -w.im;
                    CPX u = a[s + k], v = a[s + k + half];
                    CPX t = { v.re * w.re - v.im * w.im, v.re * w.im + v.im * w.re };
                    a[s + k].re = u.re + t.re; a[s + k].im = u.im + t.im;
                    a[s + k + half].re = u.re - t.re; a[s + k + half].im = u.im - t.im;
                }
            }
        }
    } else {
        for (int k = 0; k < n; ++k) {
            R sr = 0, si = 0;
            for (int t = 0; t < n; ++t) {
                CPX w = p->tw[(int)(((long)k * t) % n)];
                if (inv) w.im = -w.im;
                sr += a[t].re * w.re - a[t].im * w.im;
                si += a[t].re * w.im + a[t].im * w.re;
            }
            scratch[k].re = sr; scratch[k].im = si;
        }
        memcpy(a, scratch, sizeof(CPX) * n);
    }
}

/* rfft over dims (1,2) of an M x N real plane (line j = x[j*M .. j*M+M-1]), halving dim1:
 * out[j*H + k], H = M/2+1 (FFTW/CUFFT `rfft(v,(1,2))`, ops.jl:26,86).  Two real lines are
 * packed into one complex FFT along dim1, then a complex FFT along dim2 per bin. */
static void FN(rfft2)(const R *x, CPX *out, int M, int N, const PLAN *pm, const PLAN *pn,
                      CPX *buf, CPX *scr) {
    const int H = M / 2 + 1;
    for (int j = 0; j < N; j += 2) {
        const int two = (j + 1 < N);
        for (int i = 0; i < M; ++i) {
            buf[i].re = x[(size_t)j * M + i];
            buf[i].im = two ? x[(size_t)(j + 1) * M + i] : (R)0;
        }
        FN(fft)(pm, buf, scr, 0);
        for (int k = 0; k < H; ++k) {
            CPX zk = buf[k], zm = buf[(M - k) % M];
            /* A = (Z[k] + conj Z[-k]) / 2 ; B = (Z[k] - conj Z[-k]) / (2i) */
            out[(size_t)j * H + k].re = (R)0.5 * (zk.re + zm.re);
            out[(size_t)j * H + k].im = (R)0.5 * (zk.im - zm.im);
            if (two) {
                out[(size_t)(j + 1) * H + k].re = (R)0.5 * (zk.im + zm.im);
                out[(size_t)(j + 1) * H + k].im = (R)0.5 * (zm.re - zk.re);
            }
        }
    }
    for (int k = 0; k < H; ++k) {
        for (int j = 0; j < N; ++j) buf[j] = out[(size_t)j * H + k];
        FN(fft)(pn, buf, scr, 0);
        for (int j = 0; j < N; ++j) out[(size_t)j * H + k] = buf[j];
    }
}

/* irfft(X, M, (1,2)) normalised by 1/(MN); X is destroyed. */
static void FN(irfft2)(CPX *X, R *x, int M, int N, const PLAN *pm, const PLAN *pn,
                       CPX *buf, CPX *scr) {
    const int H = M / 2 + 1;
    const R scale = (R)1 / ((R)M * (R)N);
    for (int k = 0; k < H; ++k) {
        for (int j = 0; j < N; ++j) buf[j] = X[(size_t)j * H + k];
        FN(fft)(pn, buf, scr, 1);
        for (int j = 0; j < N; ++j) X[(size_t)j * H + k] = buf[j];
    }
    for (int j = 0; j < N; j += 2) {
        const int two = (j + 1 < N);
        const CPX *A = X + (size_t)j * H;
        const CPX *Bv = two ? X + (size_t)(j + 1) * H : NULL;
        for (int k = 0; k < M; ++k) {
            /* Hermitian extension; c2r ignores the imaginary part of the DC and Nyquist bins */
            CPX a, b = { 0, 0 };
            if (k < H) { a = A[k]; if (two) b = Bv[k]; }
            else { a.re = A[M - k].re; a.im = -A[M - k].im;
                   if (two) { b.re = Bv[M - k].re; b.im = -Bv[M - k].im; } }
            if (k == 0 || (2 * k == M)) { a.im = 0; b.im = 0; }
            buf[k].re = a.re - b.im;
            buf[k].im = a.im + b.re;
        }
        FN(fft)(pm, buf, scr, 1);
        for (int i = 0; i < M; ++i) {
            x[(size_t)j * M + i] = buf[i].re * scale;
            if (two) x[(size_t)(j + 1) * M + i] = buf[i].im * scale;
        }
    }
}

/* H^T(y): out[i,j] = sum_{a,b} h[a,b] y[i+a-padd, j+b-padr] (0-based, periodic). ops.jl:72-81 */
static void FN(ht_plane)(const R *y, R *out, int M, int N, const R *h, int kh, int kw) {
    const int padd = (kh - 1) / 2, padr = (kw - 1) / 2;
    for (size_t t = 0; t < (size_t)M * N; ++t) out[t] = 0;
    for (int b = 0; b < kw; ++b) {
        for (int a = 0; a < kh; ++a) {
            const R w = h[(size_t)b * kh + a];
            if (w == (R)0) continue;
            const int di = ((a - padd) % M + M) % M;
            for (int j = 0; j < N; ++j) {
                const int jj = (((j + b - padr) % N) + N) % N;
                const R *src = y + (size_t)jj * M;
                R *dst = out + (size_t)j * M;
                const int n1 = M - di;
                for (int i = 0; i < n1; ++i) dst[i] += w * src[i + di];
                for (int i = n1; i < M; ++i) dst[i] += w * src[i + di - M];
            }
        }
    }
}

int FN(oracle_tvd_fft_)(const R *y, R *xout, int M, int N, int P, int B, const R *h, int kh,
                        int kw, R lam, R rho, int iso, int maxit, int nthreads) {
    if (M < 2 || N < 1 || P < 1 || B < 1 || maxit < 0) return -1;
    const int planes = P * B;
    const size_t MN = (size_t)M * N;
    const int H = M / 2 + 1;
    const size_t HN = (size_t)H * N;
    const int haveh = (h != NULL && kh > 0 && kw > 0);
    const R tau = lam / rho;                                   /* ops.jl:20 */
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    PLAN pm, pn;
    FN(plan_init)(&pm, M);
    FN(plan_init)(&pn, N);
    const int LMAX = (M > N ? M : N);

    /* ---- C (ops.jl:22-37) ----------------------------------------------------------- */
    R *C = (R *)malloc(sizeof(R) * HN);
    {
        R *tmp = (R *)calloc(MN, sizeof(R));
        CPX *S = (CPX *)malloc(sizeof(CPX) * HN), *Lx = (CPX *)malloc(sizeof(CPX) * HN),
            *Ly = (CPX *)malloc(sizeof(CPX) * HN);
        CPX *buf = (CPX *)malloc(sizeof(CPX) * LMAX), *scr = (CPX *)malloc(sizeof(CPX) * LMAX);
        if (haveh) {
            for (int b = 0; b < kw && b < N; ++b)
                for (int a = 0; a < kh && a < M; ++a) tmp[(size_t)b * M + a] = h[(size_t)b * kh + a];
            FN(rfft2)(tmp, S, M, N, &pm, &pn, buf, scr);
        }
        memset(tmp, 0, sizeof(R) * MN);
        tmp[0] = 1; if (N > 1) tmp[M] = -1;                     /* dx_filter ops.jl:32 */
        FN(rfft2)(tmp, Lx, M, N, &pm, &pn, buf, scr);
        memset(tmp, 0, sizeof(R) * MN);
        tmp[0] = 1; tmp[1] = -1;                                /* dy_filter ops.jl:34 */
        FN(rfft2)(tmp, Ly, M, N, &pm, &pn, buf, scr);
        for (size_t t = 0; t < HN; ++t) {
            R s2 = haveh ? S[t].re * S[t].re + S[t].im * S[t].im : (R)1;
            R lx = Lx[t].re * Lx[t].re + Lx[t].im * Lx[t].im;
            R ly = Ly[t].re * Ly[t].re + Ly[t].im * Ly[t].im;
            C[t] = (R)1 / (s2 + rho * (lx + ly));
        }
        free(tmp); free(S); free(Lx); free(Ly); free(buf); free(scr);
    }

    /* ---- state (ops.jl:46-49); z,u,Dx per plane are [2][N][M] ----------------------- */
    R *x = (R *)calloc(MN * planes, sizeof(R));
    R *Dx = (R *)calloc(2 * MN * planes, sizeof(R));
    R *z = (R *)calloc(2 * MN * planes, sizeof(R));
    R *u = (R *)calloc(2 * MN * planes, sizeof(R));
    R *nrm = iso ? (R *)calloc(MN, sizeof(R)) : NULL;

    for (int it = 0; it < maxit; ++it) {
        #pragma omp parallel
        {
            R *v = (R *)malloc(sizeof(R) * MN);
            R *hty = (R *)malloc(sizeof(R) * MN);
            CPX *V = (CPX *)malloc(sizeof(CPX) * HN);
            CPX *buf = (CPX *)malloc(sizeof(CPX) * LMAX), *scr = (CPX *)malloc(sizeof(CPX) * LMAX);
            #pragma omp for schedule(dynamic, 1)
            for (int pl = 0; pl < planes; ++pl) {
                const R *yp = y + MN * pl;
                R *xp = x + MN * pl;
                const R *z1 = z + 2 * MN * pl, *z2 = z1 + MN;
                const R *u1 = u + 2 * MN * pl, *u2 = u1 + MN;
                /* H^T(y), re-evaluated each iteration as in ops.jl:86 */
                if (haveh) FN(ht_plane)(yp, hty, M, N, h, kh, kw);
                else memcpy(hty, yp, sizeof(R) * MN);
                /* v = H^T y + rho * D^T(z - u)   (ops.jl:63,65,86) */
                for (int j = 0; j < N; ++j) {
                    const int jn = (j + 1) % N;
                    for (int i = 0; i < M; ++i) {
                        const int in = (i + 1) % M;
                        R w1 = z1[(size_t)j * M + i] - u1[(size_t)j * M + i];
                        R w1n = z1[(size_t)jn * M + i] - u1[(size_t)jn * M + i];
                        R w2 = z2[(size_t)j * M + i] - u2[(size_t)j * M + i];
                        R w2n = z2[(size_t)j * M + in] - u2[(size_t)j * M + in];
                        v[(size_t)j * M + i] = hty[(size_t)j * M + i] + rho * ((w1 - w1n) + (w2 - w2n));
                    }
                }
                FN(rfft2)(v, V, M, N, &pm, &pn, buf, scr);
                for (size_t t = 0; t < HN; ++t) { V[t].re *= C[t]; V[t].im *= C[t]; }
                FN(irfft2)(V, xp, M, N, &pm, &pn, buf, scr);
                /* D(x)  (ops.jl:62,64,87) */
                R *d1 = Dx + 2 * MN * pl, *d2 = d1 + MN;
                for (int j = 0; j < N; ++j) {
                    const int jp = (j + N - 1) % N;
                    for (int i = 0; i < M; ++i) {
                        const int ip = (i + M - 1) % M;
                        d1[(size_t)j * M + i] = xp[(size_t)j * M + i] - xp[(size_t)jp * M + i];
                        d2[(size_t)j * M + i] = xp[(size_t)j * M + i] - xp[(size_t)j * M + ip];
                    }
                }
            }
            free(v); free(hty); free(V); free(buf); free(scr);
        }
        /* prox + dual (ops.jl:89-91) */
        if (!iso) {
            #pragma omp parallel for schedule(static)
            for (long t = 0; t < (long)(2 * MN * planes); ++t) {
                R s = Dx[t] + u[t];
                R a = (s < 0 ? -s : s) - tau;
                R sg = (s > 0) - (s < 0);
                R zt = sg * (a > 0 ? a : (R)0);
                z[t] = zt;
                u[t] = u[t] + Dx[t] - zt;
            }
        } else {
            #pragma omp parallel for schedule(static)
            for (long q = 0; q < (long)MN; ++q) {
                R acc = 0;
                for (int pl = 0; pl < planes; ++pl)
                    for (int c = 0; c < 2; ++c) {
                        R s = Dx[2 * MN * pl + c * MN + q] + u[2 * MN * pl + c * MN + q];
                        acc += s * s;
                    }
                nrm[q] = (R)sqrt((double)acc);
            }
            #pragma omp parallel for schedule(static)
            for (long t = 0; t < (long)(2 * MN * planes); ++t) {
                const long q = t % (long)MN;
                R s = Dx[t] + u[t];
                R f = (R)1 - tau / nrm[q];
                f = (f != f) ? f : (f > 0 ? f : (R)0);        /* Julia max propagates NaN */
                R zt = f * s;
                z[t] = zt;
                u[t] = u[t] + Dx[t] - zt;
            }
        }
    }
    memcpy(xout, x, sizeof(R) * MN * planes);                 /* ops.jl:93 (layout is P-major) */
    free(x); free(Dx); free(z); free(u); free(nrm); free(C);
    FN(plan_free)(&pm);
    FN(plan_free)(&pn);
    return 0;
}

#undef CPX
#undef PLAN
#undef FN
#undef CAT
#undef CAT_
