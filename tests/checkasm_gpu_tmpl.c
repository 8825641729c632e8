/*
 * checkasm_gpu_tmpl.c -- per-bitdepth body of the differential harness.
 * Included twice from checkasm_gpu.c with BITDEPTH 8 / 16.
 *
 * Mirrors the reference's checkasm iteration spaces
 * (tests/checkasm/mc.c:58-723, ipred.c:77-283, itx.c:243-318): every
 * function pointer of the GPU tables is called on the same pseudo-random
 * inputs as the oracle's entry, outputs compared byte-exactly including an
 * 8-pixel guard band (checkasm.c:963-1032) and, for itx, the zeroed
 * coefficient buffer (itx.c:294-295).
 */
#if BITDEPTH == 8
#define pixel uint8_t
#define coef int16_t
#define BD(x) x##_8bpc
#define HBD_ARG(v)
#define BDMAX_RAND() 0xff
#else
#define pixel uint16_t
#define coef int32_t
#define BD(x) x##_16bpc
#define HBD_ARG(v) , v
#define BDMAX_RAND() ((rnd() & 1) ? 0x3ff : 0xfff)
#endif

typedef struct {
    pixel *buf, *p;   /* p = origin inside the guard band */
    ptrdiff_t stride; /* bytes */
    int w, h;
} BD(Rect);

static BD(Rect) BD(rect_alloc)(int w, int h) {
    BD(Rect) r;
    const int pw = ((w + 16) * (int)sizeof(pixel) + 63) & ~63;
    r.stride = pw;
    r.buf = aligned_alloc(64, (size_t)pw * (h + 16));
    r.p = (pixel *)((uint8_t *)r.buf + 8 * pw + 8 * sizeof(pixel));
    r.w = w; r.h = h;
    return r;
}
static void BD(rect_clear)(BD(Rect) *r) { memset(r->buf, 0x99, (size_t)r->stride * (r->h + 16)); }
static int BD(rect_eq)(const BD(Rect) *a, const BD(Rect) *b) {
    return !memcmp(a->buf, b->buf, (size_t)a->stride * (a->h + 16));
}
static void BD(rect_fill)(BD(Rect) *a, BD(Rect) *b, int w, int h, int bdmax) {
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const pixel v = rnd() & bdmax;
            a->p[y * (a->stride / sizeof(pixel)) + x] = v;
            b->p[y * (b->stride / sizeof(pixel)) + x] = v;
        }
}


static void BD(check_mc)(void) {
    BD(Dav1dMCDSPContext) ref, gpu;
    BD(oracle_mc_dsp_init)(&ref);
    BD(dav1d_mc_dsp_init)(&gpu);
    pixel *src_buf = malloc(sizeof(pixel) * 263 * 263);
    BD(Rect) c_dst = BD(rect_alloc)(128, 128), a_dst = BD(rect_alloc)(128, 128);
    int16_t *ct = malloc(2 * 128 * 128), *at = malloc(2 * 128 * 128);
    int16_t *tmp[2] = { malloc(2 * 128 * 128), malloc(2 * 128 * 128) };
    uint8_t *mask = malloc(128 * 128), *cm = malloc(128 * 128), *am = malloc(128 * 128);

    /* mc (put), tests/checkasm/mc.c:58-112 */
    for (int f = 0; f < DGPU_N_2D_FILTERS; f++)
        for (int w = 2; w <= 128; w <<= 1)
            for (int mxy = 0; mxy < 4; mxy++) {
                const int h_min = w <= 32 ? 2 : w / 4, h_max = imax(imin(w * 4, 128), 32);
                int hi = 0;
                for (int h = h_min; h <= h_max; h = mc_h_next(h), hi++) {
                    /* quick: every (filter, w, h) cell once, the sub-pel case rotating */
                    if (g_quick && ((f + hi + w) & 3) != mxy) continue;
                    const int mx = (mxy & 1) ? rnd() % 15 + 1 : 0, my = (mxy & 2) ? rnd() % 15 + 1 : 0;
                    const int bdmax = BDMAX_RAND();
                    for (int i = 0; i < 135 * 135; i++) src_buf[i] = rnd() & bdmax;
                    const pixel *src = src_buf + 135 * 3 + 3;
                    BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                    ref.mc[f](c_dst.p, c_dst.stride, src, 135 * sizeof(pixel), w, h, mx, my HBD_ARG(bdmax));
                    gpu.mc[f](a_dst.p, a_dst.stride, src, 135 * sizeof(pixel), w, h, mx, my HBD_ARG(bdmax));
                    report("mc", BD(rect_eq)(&c_dst, &a_dst), "f%d w%d h%d mx%d my%d", f, w, h, mx, my);
                }
            }
    /* mct (prep) with the worst-case corner pattern, mc.c:114-167 */
    for (int f = 0; f < DGPU_N_2D_FILTERS; f++)
        for (int w = 4; w <= 128; w <<= 1)
            for (int mxy = 0; mxy < 4; mxy++)
                for (int h = imax(w / 4, 4), hi = 0; h <= imin(w * 4, 128); h <<= 1, hi++) {
                    if (g_quick && ((f + hi + w) & 3) != mxy) continue;
                    const int mx = (mxy & 1) ? rnd() % 15 + 1 : 0, my = (mxy & 2) ? rnd() % 15 + 1 : 0;
                    const int bdmax = BDMAX_RAND();
                    static const int8_t pat[8] = { -1, 0, -1, 0, 0, -1, 0, -1 };
                    const int sign = -(rnd() & 1);
                    for (int y = 0; y < 135; y++)
                        for (int x = 0; x < 135; x++)
                            src_buf[135 * y + x] = ((x | y) < 8 ? (pat[x] ^ pat[y] ^ sign) : (int)rnd()) & bdmax;
                    const pixel *src = src_buf + 135 * 3 + 3;
                    memset(ct, 0x55, 2 * 128 * 128); memset(at, 0x55, 2 * 128 * 128);
                    ref.mct[f](ct, src, 135 * sizeof(pixel), w, h, mx, my HBD_ARG(bdmax));
                    gpu.mct[f](at, src, 135 * sizeof(pixel), w, h, mx, my HBD_ARG(bdmax));
                    report("mct", !memcmp(ct, at, 2 * 128 * 128), "f%d w%d h%d mx%d my%d", f, w, h, mx, my);
                }
    /* scaled put / prep, mc.c:169-276 */
    for (int f = 0; f < DGPU_N_2D_FILTERS; f++)
        for (int w = 2; w <= 128; w <<= 1)
            for (int p = 0; p < 3; p++) {
                const int h_min = w <= 32 ? 2 : w / 4, h_max = imax(imin(w * 4, 128), 32);
                int hi = 0;
                for (int h = h_min; h <= h_max; h = mc_h_next(h), hi++) {
                    /* quick: every (filter, w, h) cell once, the dy kind rotating */
                    if (g_quick && (f + hi + w) % 3 != p) continue;
                    const int mx = rnd() % 1024, my = rnd() % 1024, dx = rnd() % 2048 + 1;
                    const int dy = !p ? (int)(rnd() % 2048 + 1) : p << 10;
                    const int bdmax = BDMAX_RAND();
                    for (int i = 0; i < 263 * 263; i++) src_buf[i] = rnd() & bdmax;
                    const pixel *src = src_buf + 263 * 3 + 3;
                    BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                    ref.mc_scaled[f](c_dst.p, c_dst.stride, src, 263 * sizeof(pixel), w, h, mx, my, dx, dy HBD_ARG(bdmax));
                    gpu.mc_scaled[f](a_dst.p, a_dst.stride, src, 263 * sizeof(pixel), w, h, mx, my, dx, dy HBD_ARG(bdmax));
                    report("mc_scaled", BD(rect_eq)(&c_dst, &a_dst), "f%d w%d h%d dy%d", f, w, h, dy);
                    if (w >= 4 && h >= imax(w / 4, 4) && h <= imin(w * 4, 128)) {
                        memset(ct, 0x55, 2 * 128 * 128); memset(at, 0x55, 2 * 128 * 128);
                        ref.mct_scaled[f](ct, src, 263 * sizeof(pixel), w, h, mx, my, dx, dy HBD_ARG(bdmax));
                        gpu.mct_scaled[f](at, src, 263 * sizeof(pixel), w, h, mx, my, dx, dy HBD_ARG(bdmax));
                        report("mct_scaled", !memcmp(ct, at, 2 * 128 * 128), "f%d w%d h%d dy%d", f, w, h, dy);
                    }
                }
            }
    /* compound blends on real mct[SHARP] output, mc.c:278-445 */
    for (int kind = 0; kind < 6; kind++)
        for (int w = 4; w <= 128; w <<= 1)
            for (int h = imax(w / 4, 4); h <= imin(w * 4, 128); h <<= 1) {
                const int bdmax = BDMAX_RAND();
                for (int i = 0; i < 2; i++) {
                    for (int k = 0; k < 135 * 135; k++) src_buf[k] = rnd() & bdmax;
                    ref.mct[DGPU_FILTER_2D_8TAP_SHARP](tmp[i], src_buf + 135 * 3 + 3, 135 * sizeof(pixel),
                                                      128, 128, 8, 8 HBD_ARG(bdmax));
                }
                for (int i = 0; i < 128 * 128; i++) mask[i] = rnd() % 65;
                BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                const char *nm;
                int ok;
                if (kind == 0) {
                    nm = "avg";
                    ref.avg(c_dst.p, c_dst.stride, tmp[0], tmp[1], w, h HBD_ARG(bdmax));
                    gpu.avg(a_dst.p, a_dst.stride, tmp[0], tmp[1], w, h HBD_ARG(bdmax));
                    ok = BD(rect_eq)(&c_dst, &a_dst);
                } else if (kind == 1) {
                    nm = "w_avg";
                    const int wt = rnd() % 15 + 1;
                    ref.w_avg(c_dst.p, c_dst.stride, tmp[0], tmp[1], w, h, wt HBD_ARG(bdmax));
                    gpu.w_avg(a_dst.p, a_dst.stride, tmp[0], tmp[1], w, h, wt HBD_ARG(bdmax));
                    ok = BD(rect_eq)(&c_dst, &a_dst);
                } else if (kind == 2) {
                    nm = "mask";
                    ref.mask(c_dst.p, c_dst.stride, tmp[0], tmp[1], w, h, mask HBD_ARG(bdmax));
                    gpu.mask(a_dst.p, a_dst.stride, tmp[0], tmp[1], w, h, mask HBD_ARG(bdmax));
                    ok = BD(rect_eq)(&c_dst, &a_dst);
                } else {
                    static const char *const wn[3] = { "w_mask_444", "w_mask_422", "w_mask_420" };
                    const int i = kind - 3, ssh = i > 0, ssv = i > 1, sign = rnd() & 1;
                    nm = wn[i];
                    memset(cm, 0x77, 128 * 128); memset(am, 0x77, 128 * 128);
                    ref.w_mask[i](c_dst.p, c_dst.stride, tmp[0], tmp[1], w, h, cm, sign HBD_ARG(bdmax));
                    gpu.w_mask[i](a_dst.p, a_dst.stride, tmp[0], tmp[1], w, h, am, sign HBD_ARG(bdmax));
                    ok = BD(rect_eq)(&c_dst, &a_dst) && !memcmp(cm, am, (w >> ssh) * (h >> ssv));
                }
                report(nm, ok, "w%d h%d", w, h);
            }
    /* blend / blend_v / blend_h, mc.c:447-563 */
    {
        pixel *tb = malloc(sizeof(pixel) * 128 * 128);
        for (int kind = 0; kind < 3; kind++) {
            const int wmin = kind == 0 ? 4 : 2, wmax = kind == 1 ? 32 : kind == 0 ? 32 : 128;
            for (int w = wmin; w <= wmax; w <<= 1) {
                int hmin, hmax;
                if (kind == 0) { hmin = imax(w / 2, 4); hmax = imin(w * 2, 32); }
                else if (kind == 1) { hmin = 2; hmax = w == 2 ? 64 : 128; }
                else { hmin = w == 128 ? 4 : 2; hmax = 32; }
                for (int h = hmin; h <= hmax; h <<= 1) {
                    const int bdmax = BDMAX_RAND();
                    for (int i = 0; i < 128 * 128; i++) { tb[i] = rnd() & bdmax; mask[i] = rnd() % 65; }
                    BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                    BD(rect_fill)(&c_dst, &a_dst, w, h, bdmax);
                    if (kind == 0) {
                        ref.blend(c_dst.p, c_dst.stride, tb, w, h, mask);
                        gpu.blend(a_dst.p, a_dst.stride, tb, w, h, mask);
                    } else if (kind == 1) {
                        ref.blend_v(c_dst.p, c_dst.stride, tb, w, h);
                        gpu.blend_v(a_dst.p, a_dst.stride, tb, w, h);
                    } else {
                        ref.blend_h(c_dst.p, c_dst.stride, tb, w, h);
                        gpu.blend_h(a_dst.p, a_dst.stride, tb, w, h);
                    }
                    static const char *const bn[3] = { "blend", "blend_v", "blend_h" };
                    report(bn[kind], BD(rect_eq)(&c_dst, &a_dst), "w%d h%d", w, h);
                }
            }
        }
        free(tb);
    }
    /* warp8x8 / warp8x8t, mc.c:565-641 */
    for (int it = 0; it < (g_quick ? 16 : 128); it++) {
        int16_t abcd[4];
        const int mx = (rnd() & 0x1fff) - 0xa00, my = (rnd() & 0x1fff) - 0xa00;
        const int bdmax = BDMAX_RAND();
        for (int i = 0; i < 4; i++) abcd[i] = (rnd() & 0x1fff) - 0xa00;
        for (int i = 0; i < 15 * 15; i++) src_buf[i] = rnd() & bdmax;
        const pixel *src = src_buf + 15 * 3 + 3;
        BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
        ref.warp8x8(c_dst.p, c_dst.stride, src, 15 * sizeof(pixel), abcd, mx, my HBD_ARG(bdmax));
        gpu.warp8x8(a_dst.p, a_dst.stride, src, 15 * sizeof(pixel), abcd, mx, my HBD_ARG(bdmax));
        report("warp8x8", BD(rect_eq)(&c_dst, &a_dst), "it%d", it);
        memset(ct, 0x55, 2 * 128 * 128); memset(at, 0x55, 2 * 128 * 128);
        ref.warp8x8t(ct, 8, src, 15 * sizeof(pixel), abcd, mx, my HBD_ARG(bdmax));
        gpu.warp8x8t(at, 8, src, 15 * sizeof(pixel), abcd, mx, my HBD_ARG(bdmax));
        report("warp8x8t", !memcmp(ct, at, 2 * 8 * 8), "it%d", it);
    }
    /* emu_edge, all 15 edge cases, mc.c:643-721 */
    {
        pixel *esrc = malloc(sizeof(pixel) * 160 * 160);
        pixel *ce = malloc(sizeof(pixel) * 135 * 192), *ae = malloc(sizeof(pixel) * 135 * 192);
        for (int i = 0; i < 160 * 160; i++) esrc[i] = rnd() & ((1U << BITDEPTH) - 1);
        for (int w = 4; w <= 128; w <<= 1)
            for (int h = imax(w / 4, 4); h <= imin(w * 4, 128); h <<= 1)
                for (int edge = 0; edge < 0xf; edge++) {
                    const int bw = w + (rnd() & 7), bh = h + (rnd() & 7);
                    int x, y, iw, ih;
                    emu_offsets(&x, &y, bw, bh, &iw, &ih, edge);
                    memset(ce, 0x99, sizeof(pixel) * 135 * 192); memset(ae, 0x99, sizeof(pixel) * 135 * 192);
                    ref.emu_edge(bw, bh, iw, ih, x, y, ce, 192 * sizeof(pixel), esrc, 160 * sizeof(pixel));
                    gpu.emu_edge(bw, bh, iw, ih, x, y, ae, 192 * sizeof(pixel), esrc, 160 * sizeof(pixel));
                    report("emu_edge", !memcmp(ce, ae, sizeof(pixel) * 135 * 192), "w%d h%d edge%d", bw, bh, edge);
                }
        free(esrc); free(ce); free(ae);
    }
    /* resize, mc.c:723-776 */
    {
        pixel *rsrc = malloc(sizeof(pixel) * 512 * 64);
        BD(Rect) cr = BD(rect_alloc)(1024, 64), ar = BD(rect_alloc)(1024, 64);
        for (int it = 0; it < (g_quick ? 4 : 16); it++) {
            const int bdmax = BDMAX_RAND();
            for (int i = 0; i < 512 * 64; i++) rsrc[i] = rnd() & bdmax;
            const int w_den = 9 + (rnd() & 7);
            const int src_w = 16 + (rnd() % (512 - 16 + 1));
            const int dst_w = w_den * src_w >> 3;
            const int dx = ((src_w << 14) + (dst_w >> 1)) / dst_w;
            const int err = dst_w * dx - (src_w << 14);
            const int mx0 = ((-((dst_w - src_w) << 13) + (dst_w >> 1)) / dst_w + 128 - (err >> 1)) & 0x3fff;
            BD(rect_clear)(&cr); BD(rect_clear)(&ar);
            ref.resize(cr.p, cr.stride, rsrc, 512 * sizeof(pixel), dst_w, 64, src_w, dx, mx0 HBD_ARG(bdmax));
            gpu.resize(ar.p, ar.stride, rsrc, 512 * sizeof(pixel), dst_w, 64, src_w, dx, mx0 HBD_ARG(bdmax));
            report("resize", BD(rect_eq)(&cr, &ar), "src_w%d dst_w%d", src_w, dst_w);
        }
        free(cr.buf); free(ar.buf); free(rsrc);
    }
    free(src_buf); free(c_dst.buf); free(a_dst.buf); free(ct); free(at);
    free(tmp[0]); free(tmp[1]); free(mask); free(cm); free(am);
}

static void BD(check_ipred)(void) {
    BD(Dav1dIntraPredDSPContext) ref, gpu;
    BD(oracle_intra_pred_dsp_init)(&ref);
    BD(dav1d_intra_pred_dsp_init)(&gpu);
    BD(Rect) c_dst = BD(rect_alloc)(64, 64), a_dst = BD(rect_alloc)(64, 64);
    pixel tl_buf[257], *const tl = tl_buf + 128;
    static const uint8_t z_angles[27] = { 3, 6, 9, 14, 17, 20, 23, 26, 29, 32, 36, 39, 42, 45,
                                          48, 51, 54, 58, 61, 64, 67, 70, 73, 76, 81, 84, 87 };
    /* intra_pred, ipred.c:77-155 */
    for (int mode = 0; mode < DGPU_N_IMPL_INTRA_PRED_MODES; mode++) {
        const int bpc_lo = (mode == DGPU_FILTER_PRED && BITDEPTH == 16) ? 10 : BITDEPTH;
        const int bpc_hi = (mode == DGPU_FILTER_PRED && BITDEPTH == 16) ? 12 : BITDEPTH;
        for (int bpc = bpc_lo; bpc <= bpc_hi; bpc += 2)
            for (int w = 4; w <= (mode == DGPU_FILTER_PRED ? 32 : 64); w <<= 1)
                for (int h = imax(w / 4, 4); h <= imin(w * 4, mode == DGPU_FILTER_PRED ? 32 : 64); h <<= 1) {
                    const int iters = (mode >= DGPU_Z1_PRED && mode <= DGPU_Z3_PRED) ? (g_quick ? 5 : 20) : 1;
                    for (int it = 0; it < iters; it++) {
                        int a = 0, maxw = 0, maxh = 0;
                        if (mode >= DGPU_Z1_PRED && mode <= DGPU_Z3_PRED) {
                            a = (90 * (mode - DGPU_Z1_PRED) + z_angles[rnd() % 27]) | (rnd() & 0x600);
                            if (mode == DGPU_Z2_PRED) { maxw = z2_max_wh(w); maxh = z2_max_wh(h); }
                        } else if (mode == DGPU_FILTER_PRED) {
                            a = (rnd() % 5) | (rnd() & ~511);
                        }
                        const int bdmax = bpc == 16 ? BDMAX_RAND() : (1 << bpc) - 1;
                        for (int i = -2 * h; i <= 2 * w; i++) tl[i] = rnd() & bdmax;
                        BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                        ref.intra_pred[mode](c_dst.p, c_dst.stride, tl, w, h, a, maxw, maxh HBD_ARG(bdmax));
                        gpu.intra_pred[mode](a_dst.p, a_dst.stride, tl, w, h, a, maxw, maxh HBD_ARG(bdmax));
                        report("intra_pred", BD(rect_eq)(&c_dst, &a_dst), "mode%d w%d h%d a%d(0x%03x) maxw%d maxh%d",
                               mode, w, h, a & 511, a & 0x600, maxw, maxh);
                    }
                }
    }
    /* cfl_ac, ipred.c:157-205 */
    {
        int16_t cac[32 * 32], aac[32 * 32];
        pixel luma[32 * 32];
        for (int layout = 1; layout <= 3; layout++) {
            const int ssv = layout == 1, ssh = layout != 3;
            const int hstep = 2 >> ssh, vstep = 2 >> ssv;
            for (int w = 4; w <= (32 >> ssh); w <<= 1)
                for (int h = imax(w / 4, 4); h <= imin(w * 4, 32 >> ssv); h <<= 1)
                    for (int wp = imax((w >> 2) - hstep, 0); wp >= 0; wp -= hstep)
                        for (int hp = imax((h >> 2) - vstep, 0); hp >= 0; hp -= vstep) {
                            const int bdmax = BDMAX_RAND();
                            for (int y = 0; y < (h << ssv); y++)
                                for (int x = 0; x < (w << ssh); x++) luma[y * 32 + x] = rnd() & bdmax;
                            memset(cac, 0x55, sizeof(cac)); memset(aac, 0x55, sizeof(aac));
                            ref.cfl_ac[layout - 1](cac, luma, 32 * sizeof(pixel), wp, hp, w, h);
                            gpu.cfl_ac[layout - 1](aac, luma, 32 * sizeof(pixel), wp, hp, w, h);
                            report("cfl_ac", !memcmp(cac, aac, sizeof(cac)), "layout%d w%d h%d wp%d hp%d",
                                   layout, w, h, wp, hp);
                        }
        }
    }
    /* cfl_pred, ipred.c:207-258 */
    {
        int16_t ac[32 * 32];
        for (int mode = 0; mode <= DGPU_DC_128_PRED; mode += 1 + 2 * !mode)
            for (int w = 4; w <= 32; w <<= 1)
                for (int h = imax(w / 4, 4); h <= imin(w * 4, 32); h <<= 1) {
                    const int bdmax = BDMAX_RAND();
                    const int alpha = ((rnd() & 15) + 1) * (1 - (rnd() & 2));
                    for (int i = -2 * h; i <= 2 * w; i++) tl[i] = rnd() & bdmax;
                    int avg = w * h >> 1;
                    for (int i = 0; i < w * h; i++) avg += ac[i] = rnd() & (bdmax << 3);
                    avg /= w * h;
                    for (int i = 0; i < w * h; i++) ac[i] -= avg;
                    BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                    ref.cfl_pred[mode](c_dst.p, c_dst.stride, tl, w, h, ac, alpha HBD_ARG(bdmax));
                    gpu.cfl_pred[mode](a_dst.p, a_dst.stride, tl, w, h, ac, alpha HBD_ARG(bdmax));
                    report("cfl_pred", BD(rect_eq)(&c_dst, &a_dst), "mode%d w%d h%d", mode, w, h);
                }
    }
    /* pal_pred, ipred.c:260-283 */
    {
        uint8_t idx[32 * 64];
        pixel pal[8];
        for (int w = 4; w <= 64; w <<= 1)
            for (int h = imax(w / 4, 4); h <= imin(w * 4, 64); h <<= 1) {
                const int bdmax = BDMAX_RAND();
                for (int i = 0; i < 8; i++) pal[i] = rnd() & bdmax;
                for (int i = 0; i < w * h / 2; i++) idx[i] = rnd() & 0x77;
                BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                ref.pal_pred(c_dst.p, c_dst.stride, pal, idx, w, h);
                gpu.pal_pred(a_dst.p, a_dst.stride, pal, idx, w, h);
                report("pal_pred", BD(rect_eq)(&c_dst, &a_dst), "w%d h%d", w, h);
            }
    }
    free(c_dst.buf); free(a_dst.buf);
}

static void BD(check_itx)(void) {
    BD(Dav1dInvTxfmDSPContext) ref, gpu;
    static const uint8_t order[19] = {  /* itx.c:304-310 */
        DGPU_TX_4X4, DGPU_RTX_4X8, DGPU_RTX_4X16, DGPU_RTX_8X4, DGPU_TX_8X8, DGPU_RTX_8X16,
        DGPU_RTX_8X32, DGPU_RTX_16X4, DGPU_RTX_16X8, DGPU_TX_16X16, DGPU_RTX_16X32,
        DGPU_RTX_16X64, DGPU_RTX_32X8, DGPU_RTX_32X16, DGPU_TX_32X32, DGPU_RTX_32X64,
        DGPU_RTX_64X16, DGPU_RTX_64X32, DGPU_TX_64X64 };
    static const uint8_t subsh_iters[5] = { 2, 2, 3, 5, 5 };
    coef cc[32 * 32], ac[32 * 32];
    BD(Rect) c_dst = BD(rect_alloc)(64, 64), a_dst = BD(rect_alloc)(64, 64);
    const int bpc_lo = BITDEPTH == 16 ? 10 : 8, bpc_hi = BITDEPTH == 16 ? 12 : 8;
    for (int bpc = bpc_lo; bpc <= bpc_hi; bpc += 2) {
        BD(oracle_itx_dsp_init)(&ref, bpc);
        BD(dav1d_itx_dsp_init)(&gpu, bpc);
        int n_entries = 0;
        for (int i = 0; i < 19; i++) {
            const int tx = order[i], w = txw(tx), h = txh(tx);
            const int lmax = imax(ctz(w), ctz(h)) - 2;
            for (int tp = 0; tp < DGPU_N_TX_TYPES_PLUS_LL; tp++) {
                if (!!ref.itxfm_add[tx][tp] != !!gpu.itxfm_add[tx][tp]) {
                    report("itx_table", 0, "tx%d tp%d presence differs", tx, tp);
                    continue;
                }
                if (!ref.itxfm_add[tx][tp]) continue;
                n_entries++;
                for (int subsh = 0; subsh < subsh_iters[lmax]; subsh++)
                    for (int rep = 0; rep < (g_quick ? 1 : 4); rep++) {
                        const int bdmax = (1 << bpc) - 1;
                        const int eob = gen_coefs(cc, tx, tp, w, h, subsh, bdmax, sizeof(coef));
                        memcpy(ac, cc, sizeof(cc));
                        BD(rect_clear)(&c_dst); BD(rect_clear)(&a_dst);
                        BD(rect_fill)(&c_dst, &a_dst, w, h, bdmax);
                        ref.itxfm_add[tx][tp](c_dst.p, c_dst.stride, cc, eob HBD_ARG(bdmax));
                        gpu.itxfm_add[tx][tp](a_dst.p, a_dst.stride, ac, eob HBD_ARG(bdmax));
                        const int ok = BD(rect_eq)(&c_dst, &a_dst) && !memcmp(cc, ac, sizeof(cc));
                        report("itx", ok, "%dx%d type%d subsh%d eob%d bpc%d", w, h, tp, subsh, eob, bpc);
                    }
            }
        }
        report("itx_table", n_entries == 156, "entries=%d (want 156) bpc%d", n_entries, bpc);
    }
    free(c_dst.buf); free(a_dst.buf);
}

/* init_tmp, tests/checkasm/cdef.c:42-53: under- / overflow / random fills */
static void BD(cdef_fill)(pixel *buf, int n, int bdmax) {
    const int fill_type = rnd() & 7;
    for (int i = 0; i < n; i++)
        buf[i] = fill_type == 0 ? (rnd() & 1) : fill_type == 1 ? bdmax - (rnd() & 1) : (rnd() & bdmax);
}

/* tests/checkasm/cdef.c:55-144: cdef_dir on random blocks, every fb entry
 * over strengths (pri / sec / both) x 8 directions x 16 edge sets; the whole
 * source buffer compared, so writes outside the w x h block fail too. */
static void BD(check_cdef)(void) {
    BD(Dav1dCdefDSPContext) ref, gpu;
    BD(oracle_cdef_dsp_init)(&ref);
    BD(dav1d_cdef_dsp_init)(&gpu);
    for (int i = 0; i < (g_quick ? 64 : 512); i++) {
        pixel src[64];
        const int bdmax = BDMAX_RAND();
        BD(cdef_fill)(src, 64, bdmax);
        unsigned cv = 0, av = 1;
        const int cd = ref.dir(src, 8 * sizeof(pixel), &cv HBD_ARG(bdmax));
        const int ad = gpu.dir(src, 8 * sizeof(pixel), &av HBD_ARG(bdmax));
        report("cdef_dir", cd == ad && cv == av, "dir %d/%d var %u/%u", cd, ad, cv, av);
    }
    static const int dims[3][2] = { { 8, 8 }, { 4, 8 }, { 4, 4 } };
    for (int f = 0; f < 3; f++) {
        const int w = dims[f][0], h = dims[f][1];
        for (int s = 1; s <= 3; s++)
            for (int dir = 0; dir < 8; dir++)
                for (int edges = 0; edges <= 15; edges++) {
                    pixel c_src[16 * 10 + 16], a_src[16 * 10 + 16], top_buf[16 * 2 + 16], bot_buf[16 * 2 + 16];
                    pixel left[8][2];
                    const int bdmax = BDMAX_RAND();
                    const int bd8 = (bdmax == 255 ? 8 : bdmax == 1023 ? 10 : 12) - 8;
                    BD(cdef_fill)(c_src, 16 * 10 + 16, bdmax);
                    BD(cdef_fill)(top_buf, 16 * 2 + 16, bdmax);
                    BD(cdef_fill)(bot_buf, 16 * 2 + 16, bdmax);
                    BD(cdef_fill)(&left[0][0], 16, bdmax);
                    memcpy(a_src, c_src, sizeof(c_src));
                    const int pri = s & 2 ? (1 + (int)(rnd() % 15)) << bd8 : 0;
                    const int sec = s & 1 ? 1 << ((rnd() % 3) + bd8) : 0;
                    const int damping = 3 + (rnd() & 3) + bd8 - (w == 4 || (rnd() & 1));
                    const ptrdiff_t stride = 16 * sizeof(pixel);
                    ref.fb[f](c_src + 8, stride, (const pixel (*)[2])left, top_buf + 8, bot_buf + 8, pri, sec, dir,
                              damping, edges HBD_ARG(bdmax));
                    gpu.fb[f](a_src + 8, stride, (const pixel (*)[2])left, top_buf + 8, bot_buf + 8, pri, sec, dir,
                              damping, edges HBD_ARG(bdmax));
                    report("cdef_filter", !memcmp(c_src, a_src, sizeof(c_src)),
                           "%dx%d pri %d sec %d dir %d damping %d edges %d", w, h, pri, sec, dir, damping, edges);
                }
    }
}

/* init_lpf_border, tests/checkasm/loopfilter.c:35-91: random, long flat,
 * short flat, or normal / hev lines across an edge */
static void BD(lpf_border)(pixel *dst, ptrdiff_t stride, int E, int I, int bdmax) {
    const int bd8 = (bdmax == 255 ? 8 : bdmax == 1023 ? 10 : 12) - 8, F = 1 << bd8;
    E <<= bd8; I <<= bd8;
    const int type = rnd() % 4, edge_diff = (int)(rnd() % ((E + 2) * 4)) - 2 * (E + 2);
#define CLP(v) ((pixel)imin(imax((v), 0), bdmax))
    if (type == 0) {
        for (int i = -8; i < 8; i++) dst[i * stride] = rnd() & bdmax;
    } else if (type == 1) {
        dst[-8 * stride] = rnd() & bdmax; dst[7 * stride] = rnd() & bdmax; dst[0] = rnd() & bdmax;
        dst[-stride] = CLP(dst[0] + edge_diff);
        for (int i = 1; i < 7; i++) {
            dst[-(1 + i) * stride] = CLP(dst[-stride] + (int)(rnd() % (2 * (F + 1))) - (F + 1));
            dst[i * stride] = CLP(dst[0] + (int)(rnd() % (2 * (F + 1))) - (F + 1));
        }
    } else {
        for (int i = 4; i < 8; i++) { dst[-(1 + i) * stride] = rnd() & bdmax; dst[i * stride] = rnd() & bdmax; }
        dst[0] = rnd() & bdmax;
        dst[-stride] = CLP(dst[0] + edge_diff);
        for (int i = 1; i < 4; i++) {
            if (type == 2) {
                dst[-(1 + i) * stride] = CLP(dst[-stride] + (int)(rnd() % (2 * (F + 1))) - (F + 1));
                dst[i * stride] = CLP(dst[0] + (int)(rnd() % (2 * (F + 1))) - (F + 1));
            } else {
                dst[-(1 + i) * stride] = CLP(dst[-i * stride] + (int)(rnd() % (2 * (I + 1))) - (I + 1));
                dst[i * stride] = CLP(dst[(i - 1) * stride] + (int)(rnd() % (2 * (I + 1))) - (I + 1));
            }
        }
    }
#undef CLP
}

/* tests/checkasm/loopfilter.c:93-203: every loop_filter_sb entry, every
 * filter length, random masks / levels / sharpness; the whole buffer compared */
static void BD(check_lpf)(void) {
    BD(Dav1dLoopFilterDSPContext) ref, gpu;
    BD(oracle_loop_filter_dsp_init)(&ref);
    BD(dav1d_loop_filter_dsp_init)(&gpu);
    static const char *names[4] = { "lpf_h_sb_y", "lpf_v_sb_y", "lpf_h_sb_uv", "lpf_v_sb_uv" };
    for (int e = 0; e < 4; e++) {
        const int uv = e >> 1, dir = e & 1, n_blks = uv ? 16 : 32, lf_idx = uv ? 2 : dir;
        for (int rep = 0; rep < (g_quick ? 4 : 16); rep++) {
            static pixel c_mem[128 * 16], a_mem[128 * 16];
            const int w = dir ? n_blks * 4 : 16, h = dir ? 16 : n_blks * 4;
            pixel *c_dst = dir ? c_mem + n_blks * 4 * 8 : c_mem + 8, *a_dst = dir ? a_mem + n_blks * 4 * 8 : a_mem + 8;
            const ptrdiff_t stride = w * sizeof(pixel), b4_stride = dir ? 32 : 2;
            Dav1dGpuFilterLUT lut;
            const int sharp = rnd() & 7;
            for (int level = 0; level < 64; level++) {
                int limit = level;
                if (sharp > 0) { limit >>= (sharp + 3) >> 2; limit = imin(limit, 9 - sharp); }
                limit = imax(limit, 1);
                lut.i[level] = limit;
                lut.e[level] = 2 * (level + 2) + limit;
            }
            lut.sharp[0] = (sharp + 3) >> 2;
            lut.sharp[1] = sharp ? 9 - sharp : 0xff;
            for (int i = 0; i < (uv ? 2 : 3); i++) {
                uint32_t vmask[4] = { 0 };
                uint8_t l[32 * 2][4];
                memset(l, 0, sizeof(l));
                for (int j = 0; j < n_blks; j++) {
                    const int idx = rnd() % (i + 2);
                    if (idx) vmask[idx - 1] |= 1U << j;
                    if (dir) { l[j][lf_idx] = rnd() & 63; l[j + 32][lf_idx] = rnd() & 63; }
                    else { l[j * 2][lf_idx] = rnd() & 63; l[j * 2 + 1][lf_idx] = rnd() & 63; }
                }
                const int bdmax = BDMAX_RAND();
                for (int k = 0; k < 128 * 16; k++) c_mem[k] = rnd() & bdmax;
                for (int k = 0; k < 4 * n_blks; k++) {
                    const int x = k >> 2;
                    const int L = dir ? (l[32 + x][lf_idx] ? l[32 + x][lf_idx] : l[x][lf_idx])
                                      : (l[2 * x + 1][lf_idx] ? l[2 * x + 1][lf_idx] : l[2 * x][lf_idx]);
                    BD(lpf_border)(c_dst + k * (dir ? 1 : 16), dir ? n_blks * 4 : 1, lut.e[L], lut.i[L], bdmax);
                }
                memcpy(a_mem, c_mem, sizeof(c_mem));
                const uint8_t (*lp)[4] = (const uint8_t (*)[4])&l[dir ? 32 : 1][lf_idx];
                ref.loop_filter_sb[uv][dir](c_dst, stride, vmask, lp, b4_stride, &lut, n_blks HBD_ARG(bdmax));
                gpu.loop_filter_sb[uv][dir](a_dst, stride, vmask, lp, b4_stride, &lut, n_blks HBD_ARG(bdmax));
                report(names[e], !memcmp(c_mem, a_mem, sizeof(c_mem)), "sizes<=%d rep %d bdmax %d", i, rep, bdmax);
            }
            (void)h;
        }
    }
}

/* init_tmp, tests/checkasm/looprestoration.c:40-51: a noisy checkerboard */
static void BD(lr_fill)(pixel *buf, ptrdiff_t stride_px, int w, int h, int bdmax) {
    const int noise_mask = bdmax >> 4, x_off = rnd() & 7, y_off = rnd() & 7;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            buf[y * stride_px + x] = (pixel)(((((x + x_off) ^ (y + y_off)) & 8) ? bdmax : 0) ^ (rnd() & noise_mask));
}

/* tests/checkasm/looprestoration.c:53-196: wiener 7 / 5 tap and sgr 5x5 /
 * 3x3 / mix over the 16 edge sets, random unit sizes (w <= 384, h <= 64),
 * bpc 8 or 10 / 12; the whole 448 x 64 buffer compared */
static void BD(check_lr)(void) {
    static pixel c_mem[448 * 64 + 64], a_mem[448 * 64 + 64], edge_buf[448 * 8 + 64], left[64][4];
    pixel *const c_dst = c_mem + 64, *const a_dst = a_mem + 64, *const h_edge = edge_buf + 64;
    const ptrdiff_t stride = 448 * sizeof(pixel);
    static const struct { const char *name; uint8_t idx; } sgr_data[3] = { { "sgr_5x5", 14 }, { "sgr_3x3", 10 },
                                                                          { "sgr_mix", 0 } };
    const int bpc_lo = BITDEPTH == 16 ? 10 : 8, bpc_hi = BITDEPTH == 16 ? 12 : 8;
    for (int bpc = bpc_lo; bpc <= bpc_hi; bpc += 2) {
        BD(Dav1dLoopRestorationDSPContext) ref, gpu;
        BD(oracle_loop_restoration_dsp_init)(&ref, bpc);
        BD(dav1d_loop_restoration_dsp_init)(&gpu, bpc);
        const int bdmax = (1 << bpc) - 1;
        for (int f = 0; f < 5; f++)
            for (int rep = 0; rep < (g_quick ? 1 : 3); rep++) {
                Dav1dGpuLrParams prm;
                memset(&prm, 0, sizeof(prm));
                if (f < 2) {
                    const int t = f;
                    for (int d = 0; d < 2; d++) {
                        int16_t *fl = prm.filter[d];
                        fl[0] = fl[6] = t ? 0 : (rnd() & 15) - 5;
                        fl[1] = fl[5] = (rnd() & 31) - 23;
                        fl[2] = fl[4] = (rnd() & 63) - 17;
                        fl[3] = (d ? 128 : 0) - (fl[0] + fl[1] + fl[2]) * 2;
                        if (!d && BITDEPTH != 8) fl[3] += 128;
                    }
                } else {
                    const uint16_t *sp = &dspt_sgr_params[sgr_data[f - 2].idx * 2];
                    prm.sgr.s0 = sp[0];
                    prm.sgr.s1 = sp[1];
                    prm.sgr.w0 = sp[0] ? (rnd() & 127) - 96 : 0;
                    prm.sgr.w1 = (sp[1] ? 160 - (rnd() & 127) : 33) - prm.sgr.w0;
                }
                const int base_w = 1 + (rnd() % 384), base_h = 1 + (rnd() & 63);
                BD(lr_fill)(c_mem, 448, 448, 64, bdmax);
                BD(lr_fill)(edge_buf, 448, 448, 8, bdmax);
                BD(lr_fill)(&left[0][0], 4, 4, 64, bdmax);
                for (int edges = 0; edges <= 15; edges++) {
                    const int w = (edges & DGPU_LR_HAVE_RIGHT) ? 256 : base_w;
                    const int h = (edges & DGPU_LR_HAVE_BOTTOM) ? 64 : base_h;
                    memcpy(a_mem, c_mem, sizeof(c_mem));
                    if (f < 2) {
                        ref.wiener[f](c_dst, stride, (const pixel (*)[4])left, h_edge, w, h, &prm, edges HBD_ARG(bdmax));
                        gpu.wiener[f](a_dst, stride, (const pixel (*)[4])left, h_edge, w, h, &prm, edges HBD_ARG(bdmax));
                    } else {
                        ref.sgr[f - 2](c_dst, stride, (const pixel (*)[4])left, h_edge, w, h, &prm, edges HBD_ARG(bdmax));
                        gpu.sgr[f - 2](a_dst, stride, (const pixel (*)[4])left, h_edge, w, h, &prm, edges HBD_ARG(bdmax));
                    }
                    report(f < 2 ? (f ? "wiener_5tap" : "wiener_7tap") : sgr_data[f - 2].name,
                           !memcmp(c_mem, a_mem, sizeof(c_mem)), "%dx%d edges %d bpc %d", w, h, edges, bpc);
                    memcpy(c_mem, a_mem, sizeof(c_mem));   /* both outputs equal or reported; keep going */
                }
            }
    }
}

#undef pixel
#undef coef
#undef BD
#undef HBD_ARG
#undef BDMAX_RAND
