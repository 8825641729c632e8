/*
 * dav1d_gpu.h -- C-ABI drop-in boundary for dav1d's per-block pixel
 * reconstruction DSP tables, backed by HIP kernels on MI355X (gfx950).
 *
 * Two tiers share one set of kernels:
 *
 *  1. Per-call tier (literal drop-in).  The init hooks below fill the
 *     reference's own function-pointer tables with entries that have exactly
 *     the reference signatures; each entry stages its (host) arguments to HBM,
 *     runs the HIP kernel and returns synchronously.  Replaces:
 *       Dav1dMCDSPContext        src/mc.h:116-132   (typedefs src/mc.h:38-114)
 *       Dav1dIntraPredDSPContext src/ipred.h:81-90  (typedefs src/ipred.h:44-79)
 *       Dav1dInvTxfmDSPContext   src/itx.h:42-44    (typedef  src/itx.h:37-40)
 *     init hooks  bitfn(dav1d_mc_dsp_init)         src/mc_tmpl.c:915
 *                 bitfn(dav1d_intra_pred_dsp_init) src/ipred_tmpl.c:740
 *                 bitfn(dav1d_itx_dsp_init)        src/itx_tmpl.c:200
 *     and, for the post-filters, further below:
 *       Dav1dLoopFilterDSPContext      src/loopfilter.h:39-52
 *       Dav1dCdefDSPContext            src/cdef.h:64-67
 *       Dav1dLoopRestorationDSPContext src/looprestoration.h:62-72
 *     The struct layouts below are layout-identical to the reference ones
 *     (arrays of function pointers in the same order), so a pointer to the
 *     reference's context can be passed straight in.
 *
 *  2. Batch tier (performance path).  One grid launch reconstructs a whole
 *     frame (or superblock row) of transform-block units: prediction
 *     (mc / mct+avg / intra) fused with inv_txfm_add.  All pointers are
 *     device pointers already resident in HBM; see dav1d_gpu_recon_*.
 *     Frame-tier entries also cover the intra wavefront, the batch recorder,
 *     deblocking, CDEF, loop restoration and film grain. 
 *
 * Strides are in BYTES and may be negative, as in the reference.  16bpc entry
 * points take the trailing `bitdepth_max` argument (0x3ff or 0xfff) except
 * blend*, emu_edge, cfl_ac and pal_pred (src/mc.h:96-108, src/ipred.h:56-78).
 *
 * Errors: the per-call entries return void like the reference
 * and never abort or write part of their outputs.  A HIP failure latches a
 * sticky, process-wide error (dav1d_gpu_get_error) that the caller checks at a
 * flush point, as dav1d checks its own task error latch (src/thread_task.c:
 * 453, src/lib.c:715); the failed call -- and every later one until
 * dav1d_gpu_clear_error -- then runs the entry the caller's table held before
 * the *_gpu_* hook overwrote it (the C default), or, when the library filled
 * the whole table (no previous entry), leaves its outputs untouched.  The
 * batch entry points return 0 or a negative error.
 */
#ifndef DAV1D_GPU_H
#define DAV1D_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- enums mirrored from src/levels.h / include/dav1d/headers.h -------- */

enum Dav1dGpuFilter2d {   /* src/levels.h:184-196, order horizontal,vertical */
    DGPU_FILTER_2D_8TAP_REGULAR, DGPU_FILTER_2D_8TAP_REGULAR_SMOOTH,
    DGPU_FILTER_2D_8TAP_REGULAR_SHARP, DGPU_FILTER_2D_8TAP_SHARP_REGULAR,
    DGPU_FILTER_2D_8TAP_SHARP_SMOOTH, DGPU_FILTER_2D_8TAP_SHARP,
    DGPU_FILTER_2D_8TAP_SMOOTH_REGULAR, DGPU_FILTER_2D_8TAP_SMOOTH,
    DGPU_FILTER_2D_8TAP_SMOOTH_SHARP, DGPU_FILTER_2D_BILINEAR,
    DGPU_N_2D_FILTERS
};

enum Dav1dGpuIntraMode {  /* remapped IntraPredMode, src/levels.h:108-133 */
    DGPU_DC_PRED, DGPU_VERT_PRED, DGPU_HOR_PRED, DGPU_LEFT_DC_PRED,
    DGPU_TOP_DC_PRED, DGPU_DC_128_PRED, DGPU_Z1_PRED, DGPU_Z2_PRED,
    DGPU_Z3_PRED, DGPU_SMOOTH_PRED, DGPU_SMOOTH_V_PRED, DGPU_SMOOTH_H_PRED,
    DGPU_PAETH_PRED, DGPU_FILTER_PRED, DGPU_N_IMPL_INTRA_PRED_MODES
};

enum Dav1dGpuTxfmSize {   /* RectTxfmSize, src/levels.h:44-78 */
    DGPU_TX_4X4, DGPU_TX_8X8, DGPU_TX_16X16, DGPU_TX_32X32, DGPU_TX_64X64,
    DGPU_RTX_4X8, DGPU_RTX_8X4, DGPU_RTX_8X16, DGPU_RTX_16X8, DGPU_RTX_16X32,
    DGPU_RTX_32X16, DGPU_RTX_32X64, DGPU_RTX_64X32, DGPU_RTX_4X16,
    DGPU_RTX_16X4, DGPU_RTX_8X32, DGPU_RTX_32X8, DGPU_RTX_16X64,
    DGPU_RTX_64X16, DGPU_N_RECT_TX_SIZES
};

enum Dav1dGpuTxfmType {   /* TxfmType, src/levels.h:80-100 */
    DGPU_DCT_DCT, DGPU_ADST_DCT, DGPU_DCT_ADST, DGPU_ADST_ADST,
    DGPU_FLIPADST_DCT, DGPU_DCT_FLIPADST, DGPU_FLIPADST_FLIPADST,
    DGPU_ADST_FLIPADST, DGPU_FLIPADST_ADST, DGPU_IDTX, DGPU_V_DCT, DGPU_H_DCT,
    DGPU_V_ADST, DGPU_H_ADST, DGPU_V_FLIPADST, DGPU_H_FLIPADST,
    DGPU_WHT_WHT, DGPU_N_TX_TYPES_PLUS_LL
};

/* ---- DSP table layouts, one per bitdepth ABI ----------------------------
 * DGPU_DSP_TYPES(sfx, pixel, coef, HBD) expands the reference's decl_*_fn
 * typedefs and context structs for one pixel/coef ABI (include/common/
 * bitdepth.h:36-91): sfx = 8bpc (uint8_t / int16_t, no extra argument) or
 * 16bpc (uint16_t / int32_t, trailing `int bitdepth_max`). */
#define DGPU_HBD_NONE
#define DGPU_HBD_ARG , int bitdepth_max

#define DGPU_DSP_TYPES(sfx, pixel, coef, HBD)                                  \
typedef void (*dgpu_mc_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,            \
    const pixel *src, ptrdiff_t src_stride, int w, int h, int mx, int my HBD);\
typedef void (*dgpu_mc_scaled_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,     \
    const pixel *src, ptrdiff_t src_stride, int w, int h, int mx, int my,     \
    int dx, int dy HBD);                                                      \
typedef void (*dgpu_warp8x8_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,       \
    const pixel *src, ptrdiff_t src_stride, const int16_t *abcd, int mx,      \
    int my HBD);                                                              \
typedef void (*dgpu_mct_fn_##sfx)(int16_t *tmp, const pixel *src,             \
    ptrdiff_t src_stride, int w, int h, int mx, int my HBD);                  \
typedef void (*dgpu_mct_scaled_fn_##sfx)(int16_t *tmp, const pixel *src,      \
    ptrdiff_t src_stride, int w, int h, int mx, int my, int dx, int dy HBD);  \
typedef void (*dgpu_warp8x8t_fn_##sfx)(int16_t *tmp, ptrdiff_t tmp_stride,    \
    const pixel *src, ptrdiff_t src_stride, const int16_t *abcd, int mx,      \
    int my HBD);                                                              \
typedef void (*dgpu_avg_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,           \
    const int16_t *tmp1, const int16_t *tmp2, int w, int h HBD);              \
typedef void (*dgpu_w_avg_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,         \
    const int16_t *tmp1, const int16_t *tmp2, int w, int h, int weight HBD);  \
typedef void (*dgpu_mask_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,          \
    const int16_t *tmp1, const int16_t *tmp2, int w, int h,                   \
    const uint8_t *mask HBD);                                                 \
typedef void (*dgpu_w_mask_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,        \
    const int16_t *tmp1, const int16_t *tmp2, int w, int h, uint8_t *mask,    \
    int sign HBD);                                                            \
typedef void (*dgpu_blend_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,         \
    const pixel *tmp, int w, int h, const uint8_t *mask);                     \
typedef void (*dgpu_blend_dir_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,     \
    const pixel *tmp, int w, int h);                                          \
typedef void (*dgpu_emu_edge_fn_##sfx)(intptr_t bw, intptr_t bh,              \
    intptr_t iw, intptr_t ih, intptr_t x, intptr_t y, pixel *dst,             \
    ptrdiff_t dst_stride, const pixel *src, ptrdiff_t src_stride);            \
typedef void (*dgpu_resize_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,        \
    const pixel *src, ptrdiff_t src_stride, int dst_w, int h, int src_w,      \
    int dx, int mx HBD);                                                      \
typedef struct Dav1dMCDSPContext_##sfx {                                      \
    dgpu_mc_fn_##sfx mc[DGPU_N_2D_FILTERS];                                   \
    dgpu_mc_scaled_fn_##sfx mc_scaled[DGPU_N_2D_FILTERS];                     \
    dgpu_mct_fn_##sfx mct[DGPU_N_2D_FILTERS];                                 \
    dgpu_mct_scaled_fn_##sfx mct_scaled[DGPU_N_2D_FILTERS];                   \
    dgpu_avg_fn_##sfx avg;                                                    \
    dgpu_w_avg_fn_##sfx w_avg;                                                \
    dgpu_mask_fn_##sfx mask;                                                  \
    dgpu_w_mask_fn_##sfx w_mask[3]; /* 444, 422, 420 */                       \
    dgpu_blend_fn_##sfx blend;                                                \
    dgpu_blend_dir_fn_##sfx blend_v;                                          \
    dgpu_blend_dir_fn_##sfx blend_h;                                          \
    dgpu_warp8x8_fn_##sfx warp8x8;                                            \
    dgpu_warp8x8t_fn_##sfx warp8x8t;                                          \
    dgpu_emu_edge_fn_##sfx emu_edge;                                          \
    dgpu_resize_fn_##sfx resize;                                              \
} Dav1dMCDSPContext_##sfx;                                                    \
typedef void (*dgpu_angular_ipred_fn_##sfx)(pixel *dst, ptrdiff_t stride,     \
    const pixel *topleft, int width, int height, int angle, int max_width,    \
    int max_height HBD);                                                      \
typedef void (*dgpu_cfl_ac_fn_##sfx)(int16_t *ac, const pixel *y,             \
    ptrdiff_t stride, int w_pad, int h_pad, int cw, int ch);                  \
typedef void (*dgpu_cfl_pred_fn_##sfx)(pixel *dst, ptrdiff_t stride,          \
    const pixel *topleft, int width, int height, const int16_t *ac,           \
    int alpha HBD);                                                           \
typedef void (*dgpu_pal_pred_fn_##sfx)(pixel *dst, ptrdiff_t stride,          \
    const pixel *pal, const uint8_t *idx, int w, int h);                      \
typedef struct Dav1dIntraPredDSPContext_##sfx {                               \
    dgpu_angular_ipred_fn_##sfx intra_pred[DGPU_N_IMPL_INTRA_PRED_MODES];     \
    dgpu_cfl_ac_fn_##sfx cfl_ac[3];  /* 420, 422, 444 */                      \
    dgpu_cfl_pred_fn_##sfx cfl_pred[DGPU_DC_128_PRED + 1];                    \
    dgpu_pal_pred_fn_##sfx pal_pred;                                          \
} Dav1dIntraPredDSPContext_##sfx;                                             \
typedef void (*dgpu_itxfm_fn_##sfx)(pixel *dst, ptrdiff_t dst_stride,         \
    coef *coeff, int eob HBD);                                                \
typedef struct Dav1dInvTxfmDSPContext_##sfx {                                 \
    dgpu_itxfm_fn_##sfx itxfm_add[DGPU_N_RECT_TX_SIZES][DGPU_N_TX_TYPES_PLUS_LL]; \
} Dav1dInvTxfmDSPContext_##sfx;

DGPU_DSP_TYPES(8bpc, uint8_t, int16_t, DGPU_HBD_NONE)
DGPU_DSP_TYPES(16bpc, uint16_t, int32_t, DGPU_HBD_ARG)

/* ---- per-call tier: init hooks ------------------------------------------
 * Same names and signatures as the reference's init hooks
 * (src/mc.h:134, src/ipred.h:92, src/itx.h:46): linking this library in place
 * of mc_tmpl.c / ipred_tmpl.c / itx_tmpl.c objects makes every table entry
 * GPU-backed.  The *_gpu_* variants are arch-style override hooks (the
 * mc_dsp_init_x86 pattern, src/x86/mc.h:108) for builds that keep the C
 * defaults and overwrite entries when the GPU cpu-flag is set.  Entries that
 * the reference leaves NULL (unsupported itx size/type pairs) stay NULL. */
void dav1d_mc_dsp_init_8bpc(Dav1dMCDSPContext_8bpc *c);
void dav1d_mc_dsp_init_16bpc(Dav1dMCDSPContext_16bpc *c);
void dav1d_intra_pred_dsp_init_8bpc(Dav1dIntraPredDSPContext_8bpc *c);
void dav1d_intra_pred_dsp_init_16bpc(Dav1dIntraPredDSPContext_16bpc *c);
void dav1d_itx_dsp_init_8bpc(Dav1dInvTxfmDSPContext_8bpc *c, int bpc);
void dav1d_itx_dsp_init_16bpc(Dav1dInvTxfmDSPContext_16bpc *c, int bpc);

void dav1d_mc_dsp_init_gpu_8bpc(Dav1dMCDSPContext_8bpc *c);
void dav1d_mc_dsp_init_gpu_16bpc(Dav1dMCDSPContext_16bpc *c);
void dav1d_intra_pred_dsp_init_gpu_8bpc(Dav1dIntraPredDSPContext_8bpc *c);
void dav1d_intra_pred_dsp_init_gpu_16bpc(Dav1dIntraPredDSPContext_16bpc *c);
void dav1d_itx_dsp_init_gpu_8bpc(Dav1dInvTxfmDSPContext_8bpc *c, int bpc);
void dav1d_itx_dsp_init_gpu_16bpc(Dav1dInvTxfmDSPContext_16bpc *c, int bpc);

/* ---- runtime -------------------------------------------------------------*/
/* Number of usable gfx950 devices (0 when no GPU / no HIP runtime). */
int dav1d_gpu_device_count(void);
/* Device used by the calling thread's per-call entries (default 0). */
int dav1d_gpu_set_device(int device);
/* Library build identification, e.g. "dav1d-gpu gfx950 r3". */
const char *dav1d_gpu_version(void);
/* SHA-1 of the sources the library was built from (tools/src_hash.py). */
const char *dav1d_gpu_source_hash(void);
/* Sticky error of the per-call tier: 0, or the first HIP error code (-1: no
 * device) latched since the last clear.  While it is set the per-call entries
 * do not touch the GPU (fallback entries, or no output).  clear returns the
 * previous value and re-enables the GPU path.  Test hook: the environment
 * variable DAV1D_GPU_FAIL_AFTER=n fails the (n+1)-th HIP call of the tier. */
int dav1d_gpu_get_error(void);
int dav1d_gpu_clear_error(void);
/* Diagnostics (the DGPU_BOUNDS build, tools/build_variants.sh bounds): add
 * one device buffer the calling thread's next batch launches (unit and tile
 * batches) may touch, with its size in bytes; those launches then check every
 * record, coefficient, edge and aux access against the registered buffers
 * and their planes (strict mode).  p = NULL clears the calling thread's list.
 * Product builds never read the list: callers register only when they run
 * the diagnostics build.  Returns 0.
 * (Both batch tiers read coefficient, edge and record arrays as aligned
 * 16-byte blocks: the 16-byte block holding an array's last byte must be
 * readable, as every device allocation's granularity makes it.) */
int dav1d_gpu_debug_register_buffer(const void *p, size_t bytes, int id);

/* ---- batch tier ----------------------------------------------------------
 * A batch is an array of transform-block "units" (one per inv_txfm_add call
 * the reference would make, src/recon_tmpl.c:816/1347/1574/1956/2017), each
 * carrying the prediction that precedes it in recon_b_inter/recon_b_intra
 * (src/recon_tmpl.c:1195, :1598).  Units are sorted by tx size class by the
 * producer; dav1d_gpu_recon_* launches ONE grid over all of them. */

enum Dav1dGpuPredKind {
    DGPU_PRED_NONE = 0,      /* residual only: dst += itx(coef)            */
    DGPU_PRED_INTER = 1,     /* mc put from ref0                             */
    DGPU_PRED_INTER_AVG = 2, /* mct(ref0) + mct(ref1) -> avg                 */
    DGPU_PRED_INTRA = 3,     /* intra_pred from the unit's edge array        */
    DGPU_PRED_CFL = 4,       /* chroma-from-luma: cfl_ac on the co-located
                                luma (batch cfl_luma plane) + cfl_pred with
                                the DC of the unit's edge array
                                (src/recon_tmpl.c:1380-1420)                 */
    DGPU_PRED_INTER_WAVG = 5,/* mct x2 -> w_avg with p.inter.weight (the
                                jnt_comp weight of ref0, 1..15;
                                src/mc_tmpl.c:604-620, recon_tmpl.c:1873)    */
    DGPU_PRED_INTER_MASK = 6,/* mct x2 -> mask_c with a per-pixel mask
                                0..64 from aux_pool (wedge / inter-intra
                                style compound; src/mc_tmpl.c:622-639,
                                recon_tmpl.c:1880-1900).  aux[unit] = byte
                                offset of the unit's top-left mask value,
                                row stride = the block width (bw4 * 4)     */
    DGPU_PRED_PAL = 7,       /* pal_pred (src/ipred_tmpl.c:717-730,
                                recon_tmpl.c:1233-1250): aux[unit] = byte
                                offset of a 16-byte aligned record of the
                                8 palette entries (pixels, padded to 16 B),
                                followed by the unit's packed index map
                                (two 4-bit indices per byte, low nibble
                                first, row stride w / 2)                     */
    DGPU_PRED_WARP = 8,      /* warp8x8 from p.inter.ref[0] for every 8x8 of
                                the unit (unit w, h multiples of 8;
                                src/mc_tmpl.c:758-791, recon_tmpl.c:1063-1100
                                warp_affine).  aux[unit] = byte offset of a
                                16-byte aligned record: int16 abcd[4], 8 pad
                                bytes, then per 8x8 (row-major) int16 x, y
                                (the warp source position in the ref plane:
                                dx, dy of recon_tmpl.c:1162-1167, relative
                                to pixel p.inter.src_off[0] of the plane,
                                normally 0), int16 mx >> 6, int16 my >> 6
                                (warp_affine clears their low 6 bits,
                                :1163-1167)                                  */
    DGPU_PRED_INTER_INTRA = 9,/* inter-intra: mc put from ref 0, intra_pred
                                into a tile, then blend (src/mc_tmpl.c:
                                641-653, recon_tmpl.c:1540-1580).  aux[unit]
                                = byte offset of a 16-byte record: int32
                                edge_off (topleft[0] in the edge pool),
                                uint8 mode, uint8 0, uint16 angle, int32
                                mask_off (aux_pool offset of the unit's
                                top-left mask value, stride bw4 * 4)         */
    DGPU_PRED_INTER_WMASK = 10,/* COMP_INTER_SEG luma: mct x2 -> w_mask_c
                                (src/mc_tmpl.c:683-740, recon_tmpl.c:1854),
                                ref[0] = tmp[mask_sign], ref[1] = the other;
                                p.inter.weight = mask_sign.  The unit WRITES
                                its part of the block's seg mask at the chroma
                                layout's resolution (cfl_ss below): aux[unit]
                                = aux_pool offset of the unit's top-left mask
                                value, row stride (bw4 * 4) >> ss_hor.  The
                                block's chroma units are INTER_MASK units on
                                that mask (recon_tmpl.c:1900); they may share
                                the batch: WMASK units run in the second
                                launch, which completes first               */
    DGPU_PRED_INTER_OBMC = 11,/* overlapped block MC (obmc(), recon_tmpl.c:
                                1071-1133): mc put from ref 0, then for every
                                neighbour prediction overlapping the unit the
                                neighbour's put (the lap call) blended in:
                                blend_h for the ones above, then blend_v for
                                the ones to the left (src/mc_tmpl.c:655-681).
                                aux[unit] = offset of a 16-byte aligned record:
                                int32 n, 12 pad bytes, then n entries of 16 B:
                                  int32 src_off (ref-plane offset of the
                                    integer position of unit pixel (0, 0)
                                    under the neighbour's mv),
                                  uint8 mx, my, filter2d, ref,
                                  uint8 x0, y0, x1, y1 (the overlap, unit
                                    pixels, [x0, x1) x [y0, y1)),
                                  uint8 lap_w4, lap_h4 (the lap call's size:
                                    its filter banks, src/mc_tmpl.c:99-107),
                                  uint8 dir (0 above: mask by row; 1 left:
                                    by column),
                                  uint8 mask_off (the mask value of unit row
                                    / column i is dav1d_obmc_masks[mask_off
                                    + i]);
                                entries above first, in decode order        */
    DGPU_PRED_INTER_SCALED = 12,/* references of another size (mc() with
                                refp->p.p.w != f->cur.p.w, recon_tmpl.c:
                                1006-1060): put_8tap_scaled (one ref) or
                                prep_8tap_scaled x2 + avg / w_avg
                                (p.inter.weight 0 = avg, 1..15 = jnt weight;
                                src/mc_tmpl.c:173-328, bilinear :452-585).
                                aux[unit] = offset of a 16-byte aligned
                                record: int32 n_refs (1 or 2), 12 pad bytes,
                                then per ref 16 B: int32 src_off (ref-plane
                                offset of the integer source position of
                                unit pixel (0, 0)), uint16 mx, my (its
                                1/1024 phase, 0..1023), uint16 dx, dy (the
                                steps, 1..2048), 4 pad bytes                 */
};

/* txtp value of a prediction-only unit (no inv_txfm_add): mc-only batches */
#define DGPU_NO_RESIDUAL 0xff

/* 32 bytes, device-resident, one per transform block.
 *
 * Coefficients are stored compactly: the nzw x nzh top-left region that can
 * be non-zero (what the reference derives from eob and the scan order,
 * src/recon_tmpl.c:460-470), column-major with stride nzh -- the reference's
 * own layout (src/itx_tmpl.c:82-85) restricted to that region.  nzw == 0
 * marks the reference's DC-only call (eob == 0 with DCT_DCT,
 * src/itx_tmpl.c:53): one coefficient is stored.  WHT_WHT (lossless,
 * src/itx_tmpl.c:166-185) is a 4x4 type (tx == DGPU_TX_4X4) with nzw, nzh
 * >= 1; every kernel runs it in int32 like the reference, for coefficients
 * over the whole dequantised range. */
typedef struct Dav1dGpuUnit {
    int32_t  dst_off;     /* pixel offset of the unit's top-left in its plane  */
    int32_t  coef_off;    /* element offset into the coefficient pool        */
    uint8_t  tx;          /* Dav1dGpuTxfmSize                                */
    uint8_t  txtp;        /* Dav1dGpuTxfmType                                */
    uint8_t  plane;       /* 0 = Y, 1 = U, 2 = V                             */
    uint8_t  pred;        /* Dav1dGpuPredKind                                */
    uint8_t  nzw, nzh;    /* stored coefficient region (0 x 0 = DC-only)     */
    uint8_t  bw4, bh4;    /* prediction-block size in 4-px units: the mc
                             4-tap/8-tap bank choice uses the block w/h
                             (src/mc_tmpl.c:99-107), not the unit's          */
    union {
        struct {          /* INTER / INTER_AVG                               */
            int32_t src_off[2];      /* pixel offset in the ref plane of the
                                        unit's top-left integer position   */
            uint8_t mx[2], my[2];    /* 1/16-pel fraction 0..15              */
            uint8_t filter2d;        /* Dav1dGpuFilter2d                     */
            uint8_t ref[2];          /* reference picture slot               */
            uint8_t weight;          /* INTER_WAVG: ref0's weight 1..15      */
        } inter;
        struct {          /* INTRA                                           */
            int32_t  edge_off;       /* offset of topleft[0] in the edge pool */
            uint16_t angle;          /* angle | is_sm<<9 | filt<<10, or
                                        filter_idx for FILTER_PRED           */
            uint8_t  mode;           /* Dav1dGpuIntraMode                    */
            uint8_t  pad_;
            uint16_t max_w, max_h;   /* Z2 edge-filter limits                */
        } intra;
        struct {          /* CFL: the unit is the whole chroma block (<= 32x32) */
            int32_t  edge_off;       /* topleft[0] in the edge pool (DC)     */
            int8_t   alpha;          /* cfl_alpha[plane], -16..16            */
            uint8_t  pad_wh;         /* w_pad | h_pad << 4 (4-px units)      */
            uint8_t  mode;           /* DC source: DC / LEFT_DC / TOP_DC /
                                        DC_128 (Dav1dGpuIntraMode)           */
            uint8_t  pad_;
            int32_t  reserved_;
            int32_t  luma_off;       /* pixel offset of the co-located luma
                                        top-left in cfl_luma                  */
        } cfl;
    } p;
} Dav1dGpuUnit;

typedef struct Dav1dGpuPlane {
    void    *data;        /* device pointer to pixel (0,0); dst planes must be
                             16-byte aligned with a 16-byte multiple stride */
    int64_t  stride;      /* bytes; the unit batch and the intra wavefront
                             take strides in [0, 2^23) (24-bit row offsets),
                             else -4                                         */
    int32_t  w, h;        /* visible size (reference reads are clamped)      */
} Dav1dGpuPlane;

#define DGPU_MAX_REFS 8

typedef struct Dav1dGpuFrameBatch {
    Dav1dGpuPlane dst[3];                    /* reconstructed planes         */
    Dav1dGpuPlane ref[DGPU_MAX_REFS][3];     /* reference pictures           */
    const Dav1dGpuUnit *units;               /* device, sorted by tx class   */
    int32_t  n_units;
    int32_t  class_start[DGPU_N_RECT_TX_SIZES + 1]; /* unit ranges per class */
    const void *coef;     /* device pool: int16 (8bpc) / int32 (16bpc)       */
    const void *edges;    /* device pool of intra topleft arrays (pixels)    */
    int32_t  bitdepth_max;
    int32_t  zero_coefs;  /* 1: honour the coefficient-zeroing contract on
                             device (src/itx_tmpl.c:55/89): consumed
                             coefficients are written back as zeros          */
    Dav1dGpuPlane cfl_luma; /* luma that CFL units read (the reconstructed
                             luma of the same blocks); must not be a plane
                             this batch writes: units run unordered          */
    int32_t  cfl_ss;      /* chroma subsampling of the frame (CFL units'
                             luma, INTER_WMASK masks): ss_hor | ss_ver << 1
                             (3 = 4:2:0, 1 = 4:2:2, 0 = 4:4:4)              */
    const int32_t *aux;   /* device, one int32 per unit (by unit index): the
                             aux_pool byte offset of an INTER_MASK unit's
                             mask or a PAL unit's palette record; only those
                             kinds read it (may be NULL without them)      */
    const void *aux_pool; /* device pool of masks (u8) / palette records;
                             INTER_WMASK units write their masks into it    */
    int32_t  class_warp[DGPU_N_RECT_TX_SIZES]; /* WARP, INTER_INTRA, INTER_
                             WMASK, INTER_OBMC and INTER_SCALED units, and
                             INTER / INTER_AVG / INTER_WAVG / INTER_MASK
                             units with a DGPU_MX_CLAMP reference, at the
                             end of each class range (units sorted so);
                             they run in a second launch whose kernel
                             keeps their registers out of the main kernel.
                             64-point classes must have none; WARP units
                             need both sides >= 8                           */
} Dav1dGpuFrameBatch;

/* Per-unit emu_edge (round 5): an INTER / INTER_AVG / INTER_WAVG /
 * INTER_MASK unit sets DGPU_MX_CLAMP in mx[k] (the fraction stays in the low
 * 4 bits) when the footprint of its reference k leaves that reference plane,
 * as recon_tmpl.c's mc() decides emu_edge (src/recon_tmpl.c:986-999); its
 * src_off[k] then holds the integer position of the unit's top-left in the
 * plane as (x & 0xffff) | (y << 16), both int16, and every footprint pixel is
 * read at its position clamped to the plane's visible w x h (emu_edge_c,
 * src/mc_tmpl.c:827-875), so unpadded pictures work.  Such units go in the
 * class_warp sub-range.  A unit without the flag is read as it stands: its
 * footprint -- the unit's rectangle -3 / +4 pixels, plus up to 3 pixels
 * before and 5 after each row for the aligned row loads -- must then lie
 * inside the plane (or inside readable edge-replicated padding).
 * Round 6: the second launch's kinds take the same flag.  INTER_WMASK,
 * INTER_OBMC (its own prediction) and INTER_INTRA: DGPU_MX_CLAMP in mx[k],
 * src_off[k] = x | y << 16 as above.  An INTER_OBMC lap entry: DGPU_MX_CLAMP
 * in its mx byte and its source offset as x | y << 16.  An INTER_SCALED
 * reference record: bit 15 of its x phase, its integer origin as
 * x | y << 16.  WARP: DGPU_MX_CLAMP in mx[0] with src_off[0] = 0, the per-8x8
 * source positions being the plane's own.  Every footprint pixel is then
 * read clamped to the plane (src/recon_tmpl.c:1036-1046, :1071-1133,
 * :1168-1177).  A clamped INTER_MASK unit reading a mask an INTER_WMASK unit
 * writes must be in a later batch than its writer (both would be in the
 * second launch). */
#define DGPU_MX_CLAMP 0x80

/* Launch one frame batch on `stream` (a hipStream_t, NULL = default).
 * Returns 0 or a negative error.  Asynchronous w.r.t. the host.
 * Reference footprints are read straight from the reference planes, except
 * for DGPU_MX_CLAMP units (above), which clamp every pixel to the plane:
 * a caller either pads its reference planes (>= 80 px, dav1d's own border
 * extension) or flags the units whose footprint leaves them (every kind,
 * since round 6). */
int dav1d_gpu_recon_8bpc(const Dav1dGpuFrameBatch *b, void *stream);
int dav1d_gpu_recon_16bpc(const Dav1dGpuFrameBatch *b, void *stream);

/* ---- batch tier, superblock tiles ----------------------------------------
 * The throughput path.  A tile is one plane's rectangle of at most 64x64
 * pixels -- a superblock's luma, or its chroma -- and one workgroup
 * reconstructs it entirely, the way recon_b_inter / recon_b_intra do for
 * the blocks of one superblock (src/recon_tmpl.c:1598, :1195):
 *   1. the residual of every transform block (inv_txfm_add's two 1-D
 *      passes, src/itx_tmpl.c:40-100) into an on-chip tile,
 *   2. the prediction of every prediction block (mc once per block and
 *      reference, as recon_tmpl.c's mc() call; intra_pred / cfl / pal per
 *      block) added to it, clipped,
 *   3. one store of the finished rectangle (whole rows).
 * Every pixel of a tile must be covered by exactly one Dav1dGpuPred; tx
 * blocks need not cover the tile (no residual there).
 *
 * Records are grouped per tile (contiguous ranges), and the per-tile lane
 * bases (`lane0`) are the producer's prefix sums -- see the comments. */

typedef struct Dav1dGpuTile {   /* 48 bytes */
    int16_t  x, y;        /* top-left in the plane, pixels                   */
    uint8_t  plane;       /* 0 = Y, 1 = U, 2 = V                             */
    uint8_t  w4, h4;      /* size in 4-px units, 1..16                       */
    uint8_t  flags;       /* bit 0: the tile has WARP preds                  */
    int32_t  pred0;       /* first Dav1dGpuPred of the tile                  */
    int32_t  tx0;         /* first Dav1dGpuTx                                */
    int32_t  coef0;       /* first coefficient (element) of the tile         */
    int32_t  edge0;       /* first intra edge pixel of the tile              */
    uint16_t n_pred, n_tx;
    uint16_t n_coef;      /* coefficients of the tile (<= 4096 + n_tx)       */
    uint16_t n_edge;      /* edge pixels of the tile (<= DGPU_TILE_MAX_EDGE) */
    uint16_t lanes_tx;    /* sum of the tx records' lane counts              */
    uint16_t lanes_coop;  /* lanes of the cooperative preds, multiple of 64  */
    uint16_t lanes_task;  /* lanes of the independent-task preds             */
    uint16_t lanes_coop_used; /* cooperative lanes actually assigned (the
                             rest of lanes_coop is padding)                 */
    int32_t  reserved2_[2];
} Dav1dGpuTile;

#define DGPU_TILE_MAX_EDGE 4608   /* edge pixels staged per tile              */

/* A prediction block (or the part of one inside the tile), 32 bytes.
 *
 * Cooperative kinds (INTRA, CFL) run as a group of 2^lanes_log2 lanes
 * (edge preparation, DC sums); they come first in the tile's pred range,
 * sorted by group size, largest first, and lane0 is the group's base in
 * the cooperative section (a multiple of its size).
 *
 * Every other kind runs as independent tasks of 4 columns x R rows,
 * R = min(8, h): (w / 4) * (h / R) tasks, one per lane; lane0 is the first
 * task's lane in the task section.  WARP needs w, h multiples of 8. */
typedef struct Dav1dGpuPred {
    uint8_t  kind;        /* Dav1dGpuPredKind (NONE: residual onto the
                             existing picture)                              */
    uint8_t  x4, y4;      /* position in the tile, 4-px units                */
    uint8_t  w4, h4;      /* size, 4-px units                                */
    uint8_t  bw4, bh4;    /* size of the whole block: the mc filter bank
                             (src/mc_tmpl.c:99-107) and mask / warp record
                             strides follow it                              */
    uint8_t  lanes_log2;  /* cooperative kinds: log2 of the group size      */
    uint16_t lane0;       /* see above                                       */
    uint16_t pad_;
    union {
        struct {          /* INTER, INTER_AVG / WAVG / MASK, INTER_INTRA,
                             WARP (ref 0 only)                               */
            int16_t src_x[2], src_y[2];  /* integer position in the reference
                             plane of the pred's top-left (the block position
                             + the mv's integer part); footprints outside the
                             plane are clamped to it (emu_edge_c,
                             src/mc_tmpl.c:827-875, as recon_tmpl.c:986-999
                             applies it)                                     */
            uint8_t mx[2], my[2];        /* 1/16-pel fractions 0..15         */
            uint8_t filter2d;            /* Dav1dGpuFilter2d                 */
            uint8_t ref[2];              /* reference picture slots          */
            uint8_t weight;              /* INTER_WAVG: ref0's weight 1..15  */
            int32_t aux;      /* aux_pool byte offset: INTER_MASK the mask
                                 value of the pred's top-left (row stride
                                 bw4 * 4); WARP / INTER_INTRA their records
                                 (as in the unit batch, the pred being the
                                 unit)                                        */
        } inter;
        struct {          /* INTRA, CFL, PAL                                 */
            int32_t  edge_off;   /* topleft[0], relative to the tile's edge0  */
            uint16_t angle;      /* angle | is_sm<<9 | filt<<10, filter_idx   */
            uint8_t  mode;       /* Dav1dGpuIntraMode (CFL: its DC source)    */
            int8_t   alpha;      /* CFL: cfl_alpha, -16..16                   */
            uint16_t max_w, max_h;   /* Z2 edge-filter limits                 */
            uint8_t  cfl_pad_wh; /* CFL: w_pad | h_pad << 4                   */
            uint8_t  pad2_[3];
            int32_t  aux;        /* CFL: luma offset in cfl_luma; PAL: the
                                    aux_pool offset of its record             */
        } intra;
    } p;
} Dav1dGpuPred;

/* A transform block, 8 bytes, bit-packed:
 *   w0 = x4 | y4 << 4 | tx << 8 | txtp << 13 | nzw << 18 | nzh << 24
 *   w1 = coef_off | lane0 << 16
 * x4, y4: position in the tile (4-px units); nzw x nzh: the stored
 * coefficient region, column-major with stride nzh (0 x 0: the reference's
 * DC-only call, one coefficient; WHT_WHT: tx 4x4, nzw, nzh >= 1); coef_off: relative to the tile's coef0;
 * lane0: base of its max(w, min(h, 32)) lanes in the tile's tx section
 * (records sorted by that lane count, largest first).  Transform blocks
 * with no residual are simply absent. */
typedef struct Dav1dGpuTx {
    uint32_t w0, w1;
} Dav1dGpuTx;

typedef struct Dav1dGpuTileBatch {
    Dav1dGpuPlane dst[3];
    Dav1dGpuPlane ref[DGPU_MAX_REFS][3];   /* w / h: the clamp bounds        */
    const Dav1dGpuTile *tiles;             /* device                         */
    int32_t  n_tiles;
    int32_t  n_tiles_huge;  /* the LAST n_tiles_huge tiles hold transform
                               blocks with a 64-point side; they run in a
                               second kernel whose registers fit the 64-point
                               transforms (the first kernel has none)       */
    int32_t  bitdepth_max;
    const Dav1dGpuPred *preds;             /* device                         */
    const Dav1dGpuTx *txs;                 /* device                         */
    void    *coef;        /* int16 (8bpc) / int32 (16bpc), tile order; zeroed
                             after use when zero_coefs (src/itx_tmpl.c:55/89) */
    const void *edges;    /* intra edge pixels, tile order                    */
    const void *aux_pool; /* masks, palette / warp / inter-intra records      */
    Dav1dGpuPlane cfl_luma;
    int32_t  cfl_ss;      /* ss_hor | ss_ver << 1                             */
    int32_t  zero_coefs;
} Dav1dGpuTileBatch;

/* Launch one tile batch: one workgroup per tile.  Reference planes need 16
 * readable bytes past the end of each row (the last one included): rows are
 * fetched with aligned 16-byte loads.  Returns 0, -1 (NULL / bad counts),
 * -3 (launch failure) or -4 (misaligned planes). */
int dav1d_gpu_recon_tiles_8bpc(const Dav1dGpuTileBatch *b, void *stream);
int dav1d_gpu_recon_tiles_16bpc(const Dav1dGpuTileBatch *b, void *stream);

/* ---- intra edge preparation ---------------------------
 * Device form of bytefn(dav1d_prepare_intra_edges) (src/ipred_prepare_tmpl.c:
 * 76-204, declared src/ipred_prepare.h:78-86) for a batch of intra transform
 * blocks: each record gathers its block's edge array (top-left, top,
 * top-right, left, bottom-left, extended as the function does when edges are
 * missing) from the reconstructed picture into the unit batch's edge pool
 * and rewrites its unit's mode (the implementation index the function
 * returns) and angle (the absolute angle | the smooth / edge-filter flags of
 * recon_tmpl.c:1238-1294).  With it, dependent intra blocks chain on the
 * device: prepare the edges of one dependency level, reconstruct it with
 * dav1d_gpu_recon_*, then the next level, all on one stream. */
typedef struct Dav1dGpuIntraEdge {   /* 16 bytes */
    int32_t unit;        /* the Dav1dGpuUnit it serves: its plane, tx size
                            (tw, th), dst_off (block position) and edge_off
                            (where topleft[0] goes) are read, its
                            p.intra.mode / angle written                    */
    int16_t x4, y4;      /* block position in the plane, 4-px units          */
    int16_t w4, h4;      /* the dependent tile's end (col_end, row_end)      */
    uint8_t mode;        /* IntraPredMode as coded: DC, V, H, the six
                            directional modes, SMOOTH*, PAETH, FILTER (13)   */
    int8_t  angle;       /* angle_delta -3..3 (FILTER: the filter index)      */
    uint8_t flags;       /* DGPU_IE_* below                                   */
    uint8_t pad_;
} Dav1dGpuIntraEdge;

#define DGPU_IE_HAVE_LEFT      1   /* x4 > tile col_start                   */
#define DGPU_IE_HAVE_TOP       2   /* y4 > tile row_start                   */
#define DGPU_IE_TOP_HAS_RIGHT  4   /* EDGE_I444_TOP_HAS_RIGHT of edge_flags  */
#define DGPU_IE_LEFT_HAS_BOTTOM 8  /* EDGE_I444_LEFT_HAS_BOTTOM              */
#define DGPU_IE_FILTER_EDGE   16   /* seq_hdr->intra_edge_filter             */
#define DGPU_IE_SMOOTH        32   /* a neighbour is SMOOTH* (sm_flag)        */
#define DGPU_IE_TOP_SB_EDGE   64   /* top row from top_edge[] (the block is at
                                      a superblock's top: prefilter_toplevel_
                                      sb_edge, recon_tmpl.c:1270-1275)       */

typedef struct Dav1dGpuIntraEdgeBatch {
    Dav1dGpuPlane pic[3];       /* reconstructed picture (read)               */
    Dav1dGpuPlane top_edge[3];  /* row r = the pre-filter row above superblock
                                   row r + 1 (f->ipred_edge); may be NULL when
                                   no record sets DGPU_IE_TOP_SB_EDGE        */
    int32_t  sb_log2[3];        /* superblock height in the plane, log2 px    */
    Dav1dGpuUnit *units;        /* device, read / written                      */
    void    *edges;             /* device edge pool (written)                  */
    const Dav1dGpuIntraEdge *recs;
    int32_t  n_recs;
    int32_t  bitdepth_max;
} Dav1dGpuIntraEdgeBatch;

/* Records whose unit is neither INTRA nor CFL are skipped (a level's record
 * range may run parallel to all its units).
 * A CFL unit's record carries mode DC_PRED, angle 0, flags without the
 * filter / smooth bits (recon_tmpl.c:1393-1410); only its DC source
 * (p.cfl.mode) is written, alpha and padding stay.  Errors: -1 NULL batch or
 * buffers / negative count, -3 launch failure. */
int dav1d_gpu_prepare_intra_edges_8bpc(const Dav1dGpuIntraEdgeBatch *b, void *stream);
int dav1d_gpu_prepare_intra_edges_16bpc(const Dav1dGpuIntraEdgeBatch *b, void *stream);

/* bytefn(dav1d_backup_ipred_edge) (src/recon_tmpl.c:2162-2186): copy the last
 * pre-filter pixel row of superblock row `sby` into top_edge row `sby`, over
 * columns [x0, x0 + w) of one plane.  A run of columns rather than the whole
 * tile row, so a wavefront can back up each column as soon as the block
 * writing it is done. */
typedef struct Dav1dGpuEdgeBackup {   /* 16 bytes */
    int32_t plane, sby;
    int32_t x0, w;
} Dav1dGpuEdgeBackup;

int dav1d_gpu_backup_ipred_edge_8bpc(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs,
                                     int n_runs, void *stream);
int dav1d_gpu_backup_ipred_edge_16bpc(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs,
                                      int n_runs, void *stream);

/* ---- intra wavefront ----------------------------------
 * Dependent intra reconstruction on the device.  The caller orders the
 * units, edge records and backup runs by dependency level (a level only
 * reads pixels written by earlier levels: the left, top, top-right,
 * bottom-left and top-left edges its records read, the co-located luma of a
 * CFL unit, the top_edge columns its runs backed up); per level the driver
 * enqueues edge preparation, reconstruction (dav1d_gpu_recon_*, the level's
 * units sorted by size class) and the level's backup runs, in that order, on
 * one stream.  This replaces recon_b_intra's per-transform-block sequence
 * prepare_intra_edges -> intra_pred / cfl_pred -> itxfm_add
 * (src/recon_tmpl.c:1195-1596) for a whole frame without host round trips. */
#define DGPU_IS_FUSED 1   /* one launch per level: the reconstruction kernel
                             gathers each unit's edges itself (record i serves
                             unit i: rec_start == unit_start) and stores
                             superblock-bottom rows to top_edge as it writes
                             them; run_start / runs are then unused */

#define DGPU_IS_PERSISTENT 2   /* one launch per frame (implies FUSED): a
                                  persistent kernel whose waves take the
                                  levels' tasks in order and wait on per-level
                                  counters in `workspace` instead of launch
                                  boundaries */

#define DGPU_IS_SB 4   /* (with PERSISTENT, round 4) the wavefront per
                          superblock: one workgroup reconstructs a whole
                          superblock, its in-superblock levels separated by
                          workgroup barriers (the hand-offs stay on the CU),
                          and waits once, for the superblocks its units read
                          (one agent-scope acquire and release per
                          superblock instead of per task).  The schedule's
                          levels are then (superblock, level inside it)
                          groups, see n_sb below.  Bit-exact, but measured
                          3x slower than the dataflow form on a 4K intra
                          frame (a longer superblock chain) */

#define DGPU_IS_DEVICE_DEPS 8   /* (with PERSISTENT) dep_start / deps are device
                                   arrays, read by the kernel where they are
                                   and not checked on the host: the batch
                                   recorder's schedules, built on the device
                                   (every unit's producers in earlier tasks) */

#define DGPU_IS_LEVEL0_BATCH 16   /* (with PERSISTENT) level 0 -- units that
                                   wait for nothing: a mixed frame's inter
                                   units and first intra units -- and each
                                   following level of at least 2048 units in
                                   ordinary fused launches, one per level,
                                   ahead of the persistent kernel, whose waves
                                   then take the levels above them only (the
                                   persistent kernel pays an atomic ticket and
                                   an agent-scope release per task, which wide
                                   levels do not need) */

typedef struct Dav1dGpuIntraSchedule {
    int32_t n_levels;
    int32_t flags;               /* DGPU_IS_*                                   */
    const int32_t *unit_start;   /* host, n_levels + 1: the level's units in
                                    recon->units (contiguous)                 */
    const int32_t *class_start;  /* host, n_levels x (DGPU_N_RECT_TX_SIZES+1):
                                    size-class ranges within the level        */
    const int32_t *rec_start;    /* host, n_levels + 1: its edge records       */
    const int32_t *run_start;    /* host, n_levels + 1: its backup runs        */
    const Dav1dGpuEdgeBackup *runs;   /* device                                */
    void    *workspace;          /* device, 16-B aligned (DGPU_IS_PERSISTENT):
                                    counters + the task list                  */
    int64_t  workspace_bytes;    /* >= dav1d_gpu_intra_workspace_bytes()       */
    /* optional (DGPU_IS_PERSISTENT): the units each unit reads pixels of,
       host CSR over recon->units (producers at lower levels; device with
       DGPU_IS_DEVICE_DEPS).  Given, a
       wave waits only for the tasks holding its units' producers instead of
       the whole previous level (dataflow); NULL: level barriers.            */
    const int32_t *dep_start;    /* n_units + 1                                */
    const int32_t *deps;
    /* DGPU_IS_SB: the levels above are (superblock, level inside it)
       groups, each superblock's groups consecutive and the superblocks in an
       order where every superblock comes after those it reads (raster order
       of the frame's superblocks does); dep_start / deps are unused.        */
    int32_t n_sb;
    const int32_t *sb_level_start;   /* host, n_sb + 1: each superblock's groups */
    const int32_t *sb_dep_start;     /* host, n_sb + 1 (CSR)                     */
    const int32_t *sb_deps;          /* host: the earlier superblocks whose pixels
                                        or top_edge rows its units read          */
    /* optional (round 4): host, one byte per unit of recon->units; above
       level 0 a wave task never spans two units with different bytes.  Give
       the units' prediction kind and coded intra mode ((pred << 4 | mode),
       the order the schedule sorts them in), and each task runs one mode's
       code path instead of several one after the other.  NULL: tasks are cut
       by size only.                                                          */
    const uint8_t *task_group;
} Dav1dGpuIntraSchedule;

/* Workspace a DGPU_IS_PERSISTENT schedule needs (bytes), or -2 if the
 * schedule is inconsistent.  After the launch, int32 [1] of the workspace is
 * non-zero if a wave gave up waiting (never expected; the frame is then
 * incomplete and the call is to be treated as failed). */
int64_t dav1d_gpu_intra_workspace_bytes(const Dav1dGpuIntraSchedule *s, int n_units);

/* recon: the frame's unit batch (units in level order, class_start and
 * class_warp ignored; cfl_luma normally the reconstructed luma plane);
 * edges: pic = the same planes, units = recon->units, every record.
 * Errors: those of the three stages, -2 inconsistent schedule, -5 workspace
 * too small or misaligned. */
int dav1d_gpu_recon_intra_frame_8bpc(const Dav1dGpuFrameBatch *recon, const Dav1dGpuIntraEdgeBatch *edges,
                                     const Dav1dGpuIntraSchedule *s, void *stream);
int dav1d_gpu_recon_intra_frame_16bpc(const Dav1dGpuFrameBatch *recon, const Dav1dGpuIntraEdgeBatch *edges,
                                      const Dav1dGpuIntraSchedule *s, void *stream);

/* ---- batch recorder ----------------------------------
 * The reconstruction seam: what recon_b_inter / recon_b_intra
 * (src/recon_tmpl.c:1598, :1195) would execute per block, recorded instead
 * (one Dav1dGpuRecBlock per block and plane, one residual per coded
 * transform block, in decode order), then reconstructed on the device by
 * one flush: the recorder cuts blocks into transform units, derives each
 * intra transform block's edge record the way recon_b_intra does
 * (:1248-1294: have_left / have_top against the tile, the per-transform
 * TOP_HAS_RIGHT / LEFT_HAS_BOTTOM from the block's edge flags), schedules
 * dependency levels (inter units at level 0; intra units after every unit
 * whose pixels their edges or CfL luma read) and runs the persistent
 * wavefront.  Host C++ (csrc/recorder.hip); device buffers are the
 * recorder's own.  4:2:0 only.
 *
 * References need no padding: mc() replaces a footprint that leaves the
 * reference picture with an emu_edge copy (src/recon_tmpl.c:986-999,
 * src/mc_tmpl.c:827-875), i.e. every read is clamped to the picture.  The
 * recorder does the same per transform unit: a unit whose footprint (with
 * the 8-tap margins) is not inside ref[slot][plane].w x .h gets a clamped
 * copy of it in a device scratch plane (filled on the flush's stream
 * before the wavefront), read through reference slot DGPU_REC_EMU_SLOT,
 * which callers therefore leave unused. */
#define DGPU_REC_EMU_SLOT (DGPU_MAX_REFS - 1)
typedef struct Dav1dGpuRecorder Dav1dGpuRecorder;

typedef struct Dav1dGpuRecBlock {
    int32_t plane;           /* 0 Y, 1 U, 2 V                                  */
    int32_t x, y, w, h;      /* the prediction block, plane pixels            */
    int32_t tx;              /* its transform size (b->tx / uvtx), uniform    */
    int32_t kind;            /* DGPU_PRED_INTER / INTER_AVG / INTER_WAVG /
                                INTRA / CFL, or (with dav1d_gpu_rec_block_aux)
                                INTER_MASK / PAL / WARP / INTER_WMASK /
                                INTER_OBMC / INTER_SCALED                     */
    int32_t tile_x0, tile_y0, tile_x1, tile_y1;   /* the tile, plane pixels    */
    /* inter: the mc() call per reference (src/recon_tmpl.c:957): the
       motion vector in 1/16 plane pixels (chroma already scaled), the ref
       slot, filter_2d, and the jnt weight for INTER_WAVG                      */
    int32_t mvx[2], mvy[2];
    uint8_t ref[2], filter2d, weight;
    /* intra: the coded mode (DC..PAETH = 0..12, FILTER 13) and angle delta
       (FILTER: the filter index); CFL: alpha (its DC source is prepared
       from DC_PRED, :1395-1410), and in `mode` cfl_ac's w_pad | h_pad << 4
       (4-px units, :1372-1380; non-zero when the block overhangs the grid) */
    uint8_t mode;
    int8_t  angle;
    int8_t  cfl_alpha;
    uint8_t flags;           /* DGPU_IE_TOP_HAS_RIGHT / LEFT_HAS_BOTTOM of the
                                block (intra_edge_flags), DGPU_IE_FILTER_EDGE,
                                DGPU_IE_SMOOTH                                 */
} Dav1dGpuRecBlock;

/* width / height: the picture's (f->cur.p.w / .h).  Blocks are recorded at
 * their full size (bw4 * 4 x bh4 * 4) and must start inside the decoder's
 * block grid, the picture rounded up to 8 (4 * f->bw x 4 * f->bh); like
 * recon_b_* the recorder cuts only the part inside the grid into transform
 * units (w4 / h4, src/recon_tmpl.c:1208), whose transform blocks may run past
 * it.  dst planes must therefore be writable over the grid plus 64 px (any
 * picture from dav1d's allocator, 128-aligned, is).  Intra max_w / max_h and
 * the top-right / bottom-left availability follow the clipped block, as in
 * recon_b_intra (:1252-1266, :1296-1298). */
Dav1dGpuRecorder *dav1d_gpu_recorder_new(int bpc, int bitdepth_max, int width, int height, int device);
void dav1d_gpu_recorder_free(Dav1dGpuRecorder *r);
/* Record one block / one coded transform block.  coef: the reference's
 * coefficient layout for inv_txfm_add (int16 8bpc, int32 16bpc; column-major,
 * min(h,32) rows, min(w,32) columns, src/itx_tmpl.c:82-85); eob as the
 * decoder passes it (eob == 0 with DCT_DCT is the DC-only call).  A
 * residual must lie inside a block recorded before it.  0 or -1. */
int dav1d_gpu_rec_block(Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b);
int dav1d_gpu_rec_residual(Dav1dGpuRecorder *r, int plane, int x, int y, int tx, int txtp, int eob,
                           const void *coef);
/* A block of a kind that carries data beside its Dav1dGpuRecBlock, with that
 * data for the whole block (the recorder cuts it per unit).  Layouts, plane
 * pixels, block-relative:
 *   INTER_MASK  (mask(), src/mc_tmpl.c:622-639; wedge / seg compound):
 *               uint8 mask[h][w] 0..64; aux = NULL for a chroma block of a
 *               COMPOUND_SEG prediction: the mask the last INTER_WMASK block
 *               wrote (recon_tmpl.c:1900)
 *   PAL         (pal_pred, ipred_tmpl.c:717-730, recon_tmpl.c:1233-1250,
 *               1425-1445): pixel pal[8] then uint8 idx[h][w / 2] (two 4-bit
 *               indices per byte, low nibble first, as t->scratch.pal_idx_*)
 *   WARP        (warp_affine, recon_tmpl.c:1134-1193): int16 abcd[4], 8 pad
 *               bytes, then per 8x8 of the block (row-major) int16 x, y, mx >> 6,
 *               my >> 6 as Dav1dGpuPredKind WARP's unit record
 *   INTER_WMASK (COMPOUND_SEG luma, w_mask, recon_tmpl.c:1854): no data
 *               (weight = mask_sign); writes the seg mask its chroma blocks'
 *               INTER_MASK (aux = NULL) read
 *   INTER_OBMC  (obmc(), recon_tmpl.c:1071-1133): int32 n, 12 pad bytes, then
 *               n lap entries of 24 B: int32 mvx, mvy (the neighbour's mv,
 *               1/16 plane px), uint8 filter2d, ref, x0, y0, x1, y1 (the
 *               overlap, block px [x0, x1) x [y0, y1)), lap_w4, lap_h4 (the
 *               lap call's size, plane px / 4), dir (0 above, 1 left),
 *               mask_off (block row / column i blends with
 *               dav1d_obmc_masks[mask_off + i]), 6 pad bytes; above first
 *   INTER_SCALED (mc() of a scaled reference, recon_tmpl.c:1006-1060):
 *               int32 n_refs, 12 pad bytes, then per ref 16 B: int32 x, y
 *               (integer source position of block pixel (0, 0): pos >> 10),
 *               uint16 mx, my (pos & 1023), uint16 dx, dy (steps)
 *   INTER_INTRA (recon_b_inter's inter-intra, recon_tmpl.c:1540-1580; blocks
 *               up to 32 x 32): uint8 mask[h][w] (the ii or wedge mask), the
 *               intra mode (DC / VERT / HOR / SMOOTH after the II_ mapping)
 *               in `mode`, ref[0] / mv[0] / filter2d the put prediction; one
 *               wavefront unit predicts the whole block (its edges gathered
 *               from the picture like an intra unit's, no edge flags, no
 *               filter), its residuals are residual-only units after it
 * INTER_WMASK / OBMC / SCALED / WARP predictions run in a launch of their own
 * ahead of the wavefront (dav1d_gpu_recon_*'s second launch), cut into
 * prediction units of at most 32 x 32; their residuals are added by PRED_NONE
 * units in the wavefront.  Their reads are clamped like every other kind's:
 * mc()'s emu_edge decision per unit and reference (translation footprints
 * and OBMC laps src/recon_tmpl.c:986-999, scaled :1036-1046 with steps of
 * 1..2048, warp 15 x 15 per 8x8 :1168-1177), a footprint leaving the
 * reference being read from a clamped copy.  0 or -1. */
int dav1d_gpu_rec_block_aux(Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b, const void *aux, size_t aux_bytes);
/* Build, upload and launch everything recorded since the last flush on
 * `stream` (the recorder waits for its previous flush before reusing its
 * buffers).  dst: the picture being reconstructed (CfL reads its luma);
 * ref: reference planes for inter blocks (w / h: the picture size every
 * read is clamped to; no padding needed; slot DGPU_REC_EMU_SLOT is the
 * recorder's).  Returns 0, -1 bad arguments, or a launch error. */
int dav1d_gpu_recorder_flush(Dav1dGpuRecorder *r, const Dav1dGpuPlane dst[3],
                             const Dav1dGpuPlane ref[DGPU_MAX_REFS][3], void *stream);
/* Superblock-top edge rows, the decoder's f->ipred_edge (replaces the
 * backup bytefn(dav1d_backup_ipred_edge), src/recon_tmpl.c:2162-2186, and
 * the top_sb_edge reads of recon_b_intra / recon_b_inter, :1275-1279,
 * :1394-1398, :1492-1496, :1664-1668, :1793-1797).  With top_edge set, every
 * flush copies the last pre-filter row of each superblock row it completes
 * into top_edge[p] row sby (the row above superblock row sby + 1) as the
 * stores happen, and intra, CfL and inter-intra units at a superblock's top
 * read the row above from there (DGPU_IE_TOP_SB_EDGE), never from the
 * picture.  A decoder can then post-filter the superblock rows already
 * flushed (dav1d_filter_sbrow per row, src/decode.c:3277: deblock, CDEF and
 * LR write the picture in place) while the next rows are recorded and
 * flushed.  Rows: the plane's grid rounded up to whole superblocks wide (as
 * dav1d's sb128w * 128), one per superblock row but the last.  sb128:
 * 128-px superblocks (64 otherwise).  top_edge NULL turns it off (the
 * default: rows above superblocks are read from the picture).  0 or -1
 * (buffers too small). */
int dav1d_gpu_recorder_set_top_edge(Dav1dGpuRecorder *r, const Dav1dGpuPlane top_edge[3], int sb128);
/* Levels and units of the last flush (diagnostics). */
int dav1d_gpu_recorder_stats(const Dav1dGpuRecorder *r, int32_t *n_units, int32_t *n_levels);
/* Device time of the last flush's prep (diagnostics): upload of the
 * recording, cut, levels, sort and scatter on the recorder's own stream,
 * from the first upload to the last step, ms (HIP events); the flush waits
 * for it, so it is part of the flush's host time too.  0 or -1. */
int dav1d_gpu_recorder_prep_ms(const Dav1dGpuRecorder *r, float *ms);
/* Outcome of the last flush (waits for it): 0, -6 if its wavefront gave up
 * waiting for producers (that picture is incomplete), -3 on a HIP error.  An
 * outcome is reported once: a -6 not read here is returned by the next flush,
 * which then launches nothing and keeps its recording.  A flush also returns
 * -1 when an inter block names a reference plane that `ref` leaves NULL. */
int dav1d_gpu_recorder_status(Dav1dGpuRecorder *r);

/* ---- device-visible pictures ---------------------------
 * A Dav1dPicAllocator (include/dav1d/picture.h:107-145) whose pictures live
 * in HBM, so a decoder's reconstructed, post-filtered and output pictures
 * stay resident between the frame-tier entries above (recorder flush ->
 * deblock -> CDEF -> LR -> grain) instead of crossing PCIe.  The layouts
 * below are layout-identical to Dav1dPicture / Dav1dPicAllocator (x86-64;
 * header types kept opaque), so `Dav1dSettings.allocator` can be set from
 * dav1d_gpu_pic_allocator_init() directly.  Plane geometry is
 * dav1d_default_picture_alloc's (src/picture.c:46-83): width and height
 * aligned to 128, strides padded by DAV1D_PICTURE_ALIGNMENT when a multiple
 * of 1024, planes 64-byte aligned and the allocation padded by 64 bytes. */
typedef struct Dav1dGpuPictureParameters {   /* Dav1dPictureParameters */
    int w, h;
    int layout;                  /* enum Dav1dPixelLayout: 0 I400 .. 3 I444 */
    int bpc;
} Dav1dGpuPictureParameters;

typedef struct Dav1dGpuPicture {             /* Dav1dPicture, 272 bytes */
    void *seq_hdr, *frame_hdr;
    void *data[3];
    ptrdiff_t stride[2];
    Dav1dGpuPictureParameters p;
    struct { int64_t timestamp, duration, offset; size_t size; const uint8_t *ud_data; void *ud_ref; } m;
    void *content_light, *mastering_display, *itut_t35;
    size_t n_itut_t35;
    uintptr_t reserved[4];
    void *frame_hdr_ref, *seq_hdr_ref, *content_light_ref, *mastering_display_ref, *itut_t35_ref;
    uintptr_t reserved_ref[4];
    void *ref;
    void *allocator_data;
} Dav1dGpuPicture;

typedef struct Dav1dGpuPicAllocator {        /* Dav1dPicAllocator */
    void *cookie;
    int (*alloc_picture_callback)(Dav1dGpuPicture *pic, void *cookie);
    void (*release_picture_callback)(Dav1dGpuPicture *pic, void *cookie);
} Dav1dGpuPicAllocator;

#define DGPU_PIC_DEVICE      0   /* hipMalloc: HBM, device access only (an all-GPU pixel path) */
#define DGPU_PIC_HOST_MAPPED 1   /* page-locked host memory mapped into the device: both sides
                                    may touch the pixels (a mixed CPU / GPU decoder)          */

/* Fill `a` with callbacks allocating on `device`; released buffers are
 * pooled per size and reused (release may come from any thread).  0 or -1.
 * alloc returns 0 or -ENOMEM like dav1d's own. */
int dav1d_gpu_pic_allocator_init(Dav1dGpuPicAllocator *a, int device, int flags);
/* Free the pool (every picture must have been released).  Returns the
 * number of pictures still outstanding (0 when clean). */
int dav1d_gpu_pic_allocator_close(Dav1dGpuPicAllocator *a);
/* A picture's plane as the frame-tier entries take it (w / h visible). */
int dav1d_gpu_picture_plane(const Dav1dGpuPicture *pic, int plane, Dav1dGpuPlane *out);

/* ---- film grain ----------------------------------------
 * bitfn(dav1d_apply_grain) (src/fg_apply_tmpl.c:222-241) on the device:
 * prep (generate_grain_y / generate_grain_uv, src/filmgrain_tmpl.c:51-144;
 * generate_scaling, fg_apply_tmpl.c:41-97; the copies of planes without
 * grain) and every 32-row strip of fgy_32x32xn / fguv_32x32xn
 * (filmgrain_tmpl.c:166-420) in two launches. */
typedef struct Dav1dGpuFilmGrainData {   /* layout of Dav1dFilmGrainData,
                                            include/dav1d/headers.h:319-337 */
    unsigned seed;
    int num_y_points;
    uint8_t y_points[14][2];            /* value, scaling */
    int chroma_scaling_from_luma;
    int num_uv_points[2];
    uint8_t uv_points[2][10][2];
    int scaling_shift;
    int ar_coeff_lag;
    int8_t ar_coeffs_y[24];
    int8_t ar_coeffs_uv[2][25 + 3];
    uint64_t ar_coeff_shift;
    int grain_scale_shift;
    int uv_mult[2];
    int uv_luma_mult[2];
    int uv_offset[2];
    int overlap_flag;
    int clip_to_restricted_range;
} Dav1dGpuFilmGrainData;

#define DGPU_GRAIN_W 82
#define DGPU_GRAIN_H 73
/* scratch: int16 grain LUTs [3][73][82], then uint8 scaling LUTs [3][4096] */
#define DGPU_GRAIN_SCRATCH_BYTES (3 * DGPU_GRAIN_H * DGPU_GRAIN_W * 2 + 3 * 4096)

typedef struct Dav1dGpuFilmGrainBatch {
    Dav1dGpuPlane in[3];     /* device: the reconstructed picture (read)      */
    Dav1dGpuPlane out[3];    /* device: the output picture (planes without
                                grain are copied), distinct from `in`        */
    Dav1dGpuFilmGrainData data;
    int32_t layout;          /* DAV1D_PIXEL_LAYOUT_*: 1 I420, 2 I422, 3 I444  */
    int32_t bitdepth_max;
    int32_t is_id;           /* seq_hdr->mtrx == DAV1D_MC_IDENTITY           */
    int32_t pad_;
    void   *scratch;         /* device, DGPU_GRAIN_SCRATCH_BYTES              */
} Dav1dGpuFilmGrainBatch;

/* in[0].w / h give the picture size.  Errors: -1 NULL / bad layout /
 * missing scratch, -3 launch failure. */
int dav1d_gpu_apply_grain_8bpc(const Dav1dGpuFilmGrainBatch *b, void *stream);
int dav1d_gpu_apply_grain_16bpc(const Dav1dGpuFilmGrainBatch *b, void *stream);

/* ---- CDEF (the first post-filter) -----------------------
 * Per-call tier: Dav1dCdefDSPContext (src/cdef.h:64-67; decl_cdef_fn :53-58,
 * decl_cdef_dir_fn :60-62) with the reference's init hook name
 * bitfn(dav1d_cdef_dsp_init) (src/cdef_tmpl.c:316-331).  fb[0] 8x8 (luma and
 * 4:4:4 chroma), fb[1] 4x8 (4:2:2), fb[2] 4x4 (4:2:0).  `left` is pixel[h][2]. */
enum Dav1dGpuCdefEdgeFlags {   /* CdefEdgeFlags, src/cdef.h:36-41 */
    DGPU_CDEF_HAVE_LEFT = 1, DGPU_CDEF_HAVE_RIGHT = 2,
    DGPU_CDEF_HAVE_TOP = 4, DGPU_CDEF_HAVE_BOTTOM = 8
};
#define DGPU_CDEF_TYPES(sfx, pixel, HBD)                                       \
typedef void (*dgpu_cdef_fn_##sfx)(pixel *dst, ptrdiff_t stride,              \
    const pixel (*left)[2], const pixel *top, const pixel *bottom,            \
    int pri_strength, int sec_strength, int dir, int damping, int edges HBD); \
typedef int (*dgpu_cdef_dir_fn_##sfx)(const pixel *dst, ptrdiff_t dst_stride, \
    unsigned *var HBD);                                                       \
typedef struct Dav1dCdefDSPContext_##sfx {                                    \
    dgpu_cdef_dir_fn_##sfx dir;                                               \
    dgpu_cdef_fn_##sfx fb[3];   /* 444/luma, 422, 420 */                      \
} Dav1dCdefDSPContext_##sfx;
DGPU_CDEF_TYPES(8bpc, uint8_t, DGPU_HBD_NONE)
DGPU_CDEF_TYPES(16bpc, uint16_t, DGPU_HBD_ARG)
void dav1d_cdef_dsp_init_8bpc(Dav1dCdefDSPContext_8bpc *c);
void dav1d_cdef_dsp_init_16bpc(Dav1dCdefDSPContext_16bpc *c);
void dav1d_cdef_dsp_init_gpu_8bpc(Dav1dCdefDSPContext_8bpc *c);
void dav1d_cdef_dsp_init_gpu_16bpc(Dav1dCdefDSPContext_16bpc *c);

/* Frame tier: bytefn(dav1d_cdef_brow) (src/cdef_apply_tmpl.c:97-309) over a
 * whole frame, as dav1d_filter_sbrow_cdef (src/recon_tmpl.c:2076-2102) runs it
 * superblock row by superblock row after deblocking.  Every 8x8 block reads
 * only deblocked, pre-CDEF pixels (the reference keeps them through its
 * cdef_line / lr_bak backups, :41-89, :132-200), so the device reads `in` and
 * writes `out`, a distinct picture: filtered blocks, and every other pixel of
 * the frame's 8x8 grid copied.
 *   The grid: f->bw = ((in[0].w + 7) >> 3) << 1 by f->bh = ((in[0].h + 7) >> 3)
 * << 1 4x4 units (src/decode.c:3598-3599); blocks are 8x8 luma at even
 * (bx, by), the last one may cover 4 px past the picture as in the
 * reference, so both pictures must be readable / writable over 4 * bw by
 * 4 * bh luma pixels (and the chroma equivalent), which dav1d's picture
 * allocation (src/picture.c:49-66) guarantees; data and strides aligned to
 * 4 pixels.  Pixels outside that grid are unavailable (CDEF_HAVE_* cleared
 * at the frame edges, :106, :127, :143-181).
 *   cdef_idx: per 64x64 luma superblock, [(bh + 15) >> 4][(bw + 15) >> 4],
 * lflvl[].cdef_idx (-1: not coded, skipped).  noskip: per 8x8 luma block,
 * [bh >> 1][bw >> 1], nonzero when lflvl[].noskip_mask has either
 * of the block's two bits (:159-161, :185-189). */
typedef struct Dav1dGpuCdefFrame {
    Dav1dGpuPlane in[3];          /* device: deblocked picture (read only)   */
    Dav1dGpuPlane out[3];         /* device: output picture, distinct        */
    const int8_t *cdef_idx;       /* device                                  */
    const uint8_t *noskip;        /* device                                  */
    int32_t layout;               /* 0 I400, 1 I420, 2 I422, 3 I444          */
    int32_t bitdepth_max;
    int32_t damping;              /* frame_hdr->cdef.damping (3..6)          */
    int32_t pad_;
    uint8_t y_strength[8];        /* frame_hdr->cdef.y_strength / uv_strength */
    uint8_t uv_strength[8];
    int32_t row_start, row_end;   /* round 5: luma rows [start, end), multiples
                                     of 64: the 64x64 filter blocks of those
                                     rows only (dav1d_cdef_brow per row);
                                     0, 0: the whole frame                   */
} Dav1dGpuCdefFrame;
/* Errors: -1 NULL / bad layout / in == out / bad damping or strength / bad
 * row range, -3 launch failure, -4 misaligned planes.  in is read-only, so
 * a range may run as soon as the deblocked rows it reads exist (its rows
 * plus 2 below, 64 + 2 per superblock row). */
int dav1d_gpu_cdef_frame_8bpc(const Dav1dGpuCdefFrame *f, void *stream);
int dav1d_gpu_cdef_frame_16bpc(const Dav1dGpuCdefFrame *f, void *stream);

/* ---- deblocking loop filter --------------------------
 * Per-call tier: Dav1dLoopFilterDSPContext (src/loopfilter.h:39-52) with the
 * reference's init name bitfn(dav1d_loop_filter_dsp_init)
 * (src/loopfilter_tmpl.c:257-272): loop_filter_sb[plane 0 y / 1 uv][0 column
 * edges (h) / 1 row edges (v)].  The limit LUT is Av1FilterLUT
 * (src/lf_mask.h:35-39). */
typedef struct Dav1dGpuFilterLUT {
    uint8_t e[64];
    uint8_t i[64];
    uint64_t sharp[2];
} Dav1dGpuFilterLUT;
#define DGPU_LPF_TYPES(sfx, pixel, HBD)                                        \
typedef void (*dgpu_loopfilter_sb_fn_##sfx)(pixel *dst, ptrdiff_t stride,     \
    const uint32_t *mask, const uint8_t (*lvl)[4], ptrdiff_t lvl_stride,      \
    const Dav1dGpuFilterLUT *lut, int w HBD);                                 \
typedef struct Dav1dLoopFilterDSPContext_##sfx {                              \
    dgpu_loopfilter_sb_fn_##sfx loop_filter_sb[2][2];                         \
} Dav1dLoopFilterDSPContext_##sfx;
DGPU_LPF_TYPES(8bpc, uint8_t, DGPU_HBD_NONE)
DGPU_LPF_TYPES(16bpc, uint16_t, DGPU_HBD_ARG)
void dav1d_loop_filter_dsp_init_8bpc(Dav1dLoopFilterDSPContext_8bpc *c);
void dav1d_loop_filter_dsp_init_16bpc(Dav1dLoopFilterDSPContext_16bpc *c);
void dav1d_loop_filter_dsp_init_gpu_8bpc(Dav1dLoopFilterDSPContext_8bpc *c);
void dav1d_loop_filter_dsp_init_gpu_16bpc(Dav1dLoopFilterDSPContext_16bpc *c);

/* Frame tier: dav1d_loopfilter_sbrow_cols / _rows (src/lf_apply_tmpl.c:
 * 314-466) for every superblock row, as dav1d_filter_sbrow_deblock_cols /
 * _rows run them (src/recon_tmpl.c:2037-2069), in place, in two launches:
 * every column edge of the frame, then every row edge.  Within one pass no
 * two edges touch the same pixels (a filter of length n needs transform
 * blocks of at least n on both sides), and a superblock row's row edges
 * touch no pixel the next row's column edges read, so this order gives the
 * reference's pixels.
 *   masks: f->lf.mask, one Av1Filter per 128x128 area (src/lf_mask.h:49-56),
 * [sb128h][sb128w], AFTER the tile-edge fixups dav1d_loopfilter_sbrow_cols
 * applies to them (:327-393; host bit operations, done before upload).
 * level: f->lf.level (uint8_t[4] per 4x4 block, luma index [0] column / [1]
 * row edges; chroma [2] u / [3] v at chroma 4x4 coordinates), row stride
 * f->b4_stride entries.  Edges at the picture's left and top are not
 * filtered; rows are honoured per 64-row half that starts inside the
 * picture, columns of column edges below f->w4 (:176-210). */
typedef struct Dav1dGpuAv1Filter {   /* Av1Filter, src/lf_mask.h:49-56 */
    uint16_t filter_y[2][32][3][2];
    uint16_t filter_uv[2][32][2][2];
    int8_t cdef_idx[4];
    uint16_t noskip_mask[16][2];
} Dav1dGpuAv1Filter;
typedef struct Dav1dGpuLoopFilterFrame {
    Dav1dGpuPlane pic[3];         /* device: the picture, filtered in place  */
    const Dav1dGpuAv1Filter *masks;   /* device                              */
    const uint8_t *level;         /* device: f->lf.level                     */
    int64_t b4_stride;            /* f->b4_stride                            */
    Dav1dGpuFilterLUT lut;        /* f->lf.lim_lut                           */
    int32_t layout;               /* 0 I400, 1 I420, 2 I422, 3 I444          */
    int32_t bitdepth_max;
    int32_t filter_uv;            /* loopfilter.level_u || level_v           */
    int32_t row_start, row_end;   /* round 5: luma rows [start, end), multiples
                                     of 64 -- the superblock rows of
                                     dav1d_filter_sbrow_deblock_cols / _rows
                                     (src/recon_tmpl.c:2037-2069), chroma
                                     rows >> ss_ver; 0, 0: the whole frame   */
    int32_t pad_;
} Dav1dGpuLoopFilterFrame;
/* Errors: -1 NULL / bad layout / bad row range, -3 launch failure.  Row
 * ranges run in increasing order give the whole-frame result (a superblock
 * row's row edges never reach pixels the next row's column edges read). */
int dav1d_gpu_loopfilter_frame_8bpc(const Dav1dGpuLoopFilterFrame *f, void *stream);
int dav1d_gpu_loopfilter_frame_16bpc(const Dav1dGpuLoopFilterFrame *f, void *stream);

/* ---- loop restoration -------------------------------
 * Per-call tier: Dav1dLoopRestorationDSPContext (src/looprestoration.h:
 * 62-72) with the reference's init name bitfn(dav1d_loop_restoration_dsp_init)
 * (src/looprestoration_tmpl.c:539-558): wiener[0/1] (7-tap / 5-tap, the same
 * function in C), sgr[0] 5x5, sgr[1] 3x3, sgr[2] mix.  One restoration unit
 * stripe per call: w <= 384, h <= 64; `left` is pixel[h][4]; `lpf` holds the
 * two loop-filtered rows above (rows 0-1) and below (rows 6-7) at `stride`. */
enum Dav1dGpuLrEdgeFlags {   /* LrEdgeFlags, src/looprestoration.h:35-40 */
    DGPU_LR_HAVE_LEFT = 1, DGPU_LR_HAVE_RIGHT = 2, DGPU_LR_HAVE_TOP = 4, DGPU_LR_HAVE_BOTTOM = 8
};
typedef union Dav1dGpuLrParams {   /* LooprestorationParams, :47-53 */
    int16_t filter[2][8] __attribute__((aligned(16)));
    struct { uint32_t s0, s1; int16_t w0, w1; } sgr;
} Dav1dGpuLrParams;
#define DGPU_LR_TYPES(sfx, pixel, HBD)                                         \
typedef void (*dgpu_lr_fn_##sfx)(pixel *dst, ptrdiff_t stride,                \
    const pixel (*left)[4], const pixel *lpf, int w, int h,                   \
    const Dav1dGpuLrParams *params, int edges HBD);                           \
typedef struct Dav1dLoopRestorationDSPContext_##sfx {                         \
    dgpu_lr_fn_##sfx wiener[2];                                               \
    dgpu_lr_fn_##sfx sgr[3];                                                  \
} Dav1dLoopRestorationDSPContext_##sfx;
DGPU_LR_TYPES(8bpc, uint8_t, DGPU_HBD_NONE)
DGPU_LR_TYPES(16bpc, uint16_t, DGPU_HBD_ARG)
void dav1d_loop_restoration_dsp_init_8bpc(Dav1dLoopRestorationDSPContext_8bpc *c, int bpc);
void dav1d_loop_restoration_dsp_init_16bpc(Dav1dLoopRestorationDSPContext_16bpc *c, int bpc);
void dav1d_loop_restoration_dsp_init_gpu_8bpc(Dav1dLoopRestorationDSPContext_8bpc *c, int bpc);
void dav1d_loop_restoration_dsp_init_gpu_16bpc(Dav1dLoopRestorationDSPContext_16bpc *c, int bpc);

/* Frame tier: bytefn(dav1d_lr_sbrow) (src/lr_apply_tmpl.c:169-202, with
 * lr_sbrow :99-167 and lr_stripe :36-97) for every superblock row, as
 * dav1d_filter_sbrow_lr runs it, without super-res.  Every stripe (64 rows,
 * the first one 8 luma rows shorter) of every restoration unit reads: its
 * own rows and the 3 columns on either side from `in` (the CDEF output;
 * dav1d keeps the left ones in pre_lr_border, :150-151), the 2 rows above
 * and below the stripe from `lpf` (the deblocked, pre-CDEF picture that
 * dav1d_copy_lpf saves into lr_lpf_line, lf_apply_tmpl.c:40-174), with
 * padding() at the picture edges.  One launch; `out` is a distinct picture
 * (units that are not restored are copied).
 *   units[p]: the plane's restoration units, [unit_rows[p]][unit_cols[p]]
 * with unit_cols = max(1, (w + half) / unit_size) (the last unit takes the
 * rest, lr_sbrow's x loop) and the unit row of a superblock row chosen as
 * lr_sbrow does (:124-127); the per-128x128 lr_mask entries of dav1d map to
 * it one to one. */
typedef struct Dav1dGpuLrUnit {   /* Av1RestorationUnit, src/lf_mask.h:41-47 */
    uint8_t type;                 /* Dav1dRestorationType: 0 none, 2 wiener,
                                     3 + sgr_idx self-guided                 */
    int8_t filter_h[3];
    int8_t filter_v[3];
    int8_t sgr_weights[2];
} Dav1dGpuLrUnit;
typedef struct Dav1dGpuLrFrame {
    Dav1dGpuPlane in[3];          /* device: CDEF output (pre-LR), read      */
    Dav1dGpuPlane lpf[3];         /* device: deblocked, pre-CDEF picture     */
    Dav1dGpuPlane out[3];         /* device: restored picture, distinct      */
    const Dav1dGpuLrUnit *units[3];
    int32_t unit_rows[3], unit_cols[3];
    int32_t unit_size_log2[2];    /* restoration.unit_size[luma, chroma]     */
    int32_t layout;               /* 0 I400, 1 I420, 2 I422, 3 I444          */
    int32_t bitdepth_max;
    int32_t sb128;
    int32_t restore_planes;       /* LR_RESTORE_Y 1 | U 2 | V 4              */
    int32_t row_start, row_end;   /* round 5: luma rows [start, end), multiples
                                     of 64: the restoration stripes k =
                                     start / 64 .. end / 64 - 1 (rows
                                     64k - 8 .. 64k + 55, >> ss_ver), what
                                     dav1d_lr_sbrow filters per superblock
                                     row (src/lr_apply_tmpl.c:169-202); a
                                     range with end >= the luma height
                                     rounded up to 64 holds the last
                                     superblock row and, as there, runs
                                     every stripe from start / 64 to the
                                     picture's bottom; 0, 0: the whole
                                     frame                                   */
} Dav1dGpuLrFrame;
/* Errors: -1 NULL / bad layout / bad unit grid / bad row range, -3 launch
 * failure. */
int dav1d_gpu_lr_frame_8bpc(const Dav1dGpuLrFrame *f, void *stream);
int dav1d_gpu_lr_frame_16bpc(const Dav1dGpuLrFrame *f, void *stream);

/* Super-res: bytefn(dav1d_filter_sbrow_resize)
 * (src/recon_tmpl.c:2104-2137) for a whole frame.  Every row of every plane
 * of the post-CDEF picture is upscaled horizontally by mc.resize (resize_c,
 * src/mc_tmpl.c:877-903) into the super-res picture.  The reference resizes
 * one superblock row at a time, 8 rows (>> ss_ver) behind the CDEF; those
 * row ranges tile the picture and the filter works on one row at a time, so
 * one launch over the finished picture computes the same pixels.  in[p].w is
 * the coded width the filter clamps to, (4 * f->bw + ss_hor) >> ss_hor;
 * out[p].w the upscaled width, (f->sr_cur.p.p.w + ss_hor) >> ss_hor; in[p].h
 * the plane height.  out must not alias in.  For loop restoration after
 * super-res, upscale the deblocked picture the same way and hand it to
 * dav1d_gpu_lr_frame_* as its lpf source (backup_lpf resizes the rows it
 * keeps, src/lf_apply_tmpl.c:63-80).  Errors: -1 NULL / bad layout / bad
 * sizes, -3 launch failure. */
typedef struct Dav1dGpuResizeFrame {
    Dav1dGpuPlane in[3];          /* device: the coded-width picture, read  */
    Dav1dGpuPlane out[3];         /* device: the upscaled picture, written  */
    int32_t step[2], start[2];    /* f->resize_step / resize_start [luma, chroma] */
    int32_t layout;               /* 0 I400, 1 I420, 2 I422, 3 I444          */
    int32_t bitdepth_max;
    int32_t sb128;                /* the superblock-row walk (oracle only)   */
    int32_t pad_;
} Dav1dGpuResizeFrame;
int dav1d_gpu_resize_frame_8bpc(const Dav1dGpuResizeFrame *f, void *stream);
int dav1d_gpu_resize_frame_16bpc(const Dav1dGpuResizeFrame *f, void *stream);

/* LDS bytes per workgroup of a batch kernel (bpc 8/16; group 0: the main
 * kernel, every size up to 32x32; 1: the large sizes when built with split
 * groups; 2: a 64-point side; 3: the warp kernel; -1 otherwise).
 * Diagnostics.  Errors of dav1d_gpu_recon_*: -1 NULL batch / units, -2 bad
 * class_start / class_warp ranges, -3 launch failure, -4 misaligned planes. */
int dav1d_gpu_recon_lds_bytes(int bpc, int group);

#ifdef __cplusplus
}
#endif

#endif /* DAV1D_GPU_H */
