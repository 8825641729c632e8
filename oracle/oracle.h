/* oracle.h -- entry points of the CPU restatement (oracle/dsp_ref.c).
 * TEST INFRASTRUCTURE ONLY (see dsp_ref.c header). */
#ifndef DAV1D_ORACLE_H
#define DAV1D_ORACLE_H
#include "dav1d_gpu.h"
void oracle_mc_dsp_init_8bpc(Dav1dMCDSPContext_8bpc *c);
void oracle_mc_dsp_init_16bpc(Dav1dMCDSPContext_16bpc *c);
void oracle_intra_pred_dsp_init_8bpc(Dav1dIntraPredDSPContext_8bpc *c);
void oracle_intra_pred_dsp_init_16bpc(Dav1dIntraPredDSPContext_16bpc *c);
void oracle_itx_dsp_init_8bpc(Dav1dInvTxfmDSPContext_8bpc *c, int bpc);
void oracle_itx_dsp_init_16bpc(Dav1dInvTxfmDSPContext_16bpc *c, int bpc);
int oracle_itx_supported_8bpc(int tx, int tp);
int oracle_recon_units_8bpc(const Dav1dGpuFrameBatch *b, int u0, int u1);
int oracle_recon_units_16bpc(const Dav1dGpuFrameBatch *b, int u0, int u1);
int oracle_recon_tiles_8bpc(const Dav1dGpuTileBatch *b, int t0, int t1);
int oracle_recon_tiles_16bpc(const Dav1dGpuTileBatch *b, int t0, int t1);
int oracle_prepare_intra_edges_8bpc(const Dav1dGpuIntraEdgeBatch *b);
int oracle_prepare_intra_edges_16bpc(const Dav1dGpuIntraEdgeBatch *b);
int oracle_backup_ipred_edge_8bpc(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs, int n);
int oracle_backup_ipred_edge_16bpc(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs, int n);
int oracle_recon_intra_frame_8bpc(const Dav1dGpuFrameBatch *rb, const Dav1dGpuIntraEdgeBatch *eb,
                                  const int32_t *steps, int n_steps, const int32_t *unit_rec,
                                  const Dav1dGpuEdgeBackup *runs);
int oracle_recon_intra_frame_16bpc(const Dav1dGpuFrameBatch *rb, const Dav1dGpuIntraEdgeBatch *eb,
                                   const int32_t *steps, int n_steps, const int32_t *unit_rec,
                                   const Dav1dGpuEdgeBackup *runs);
int oracle_prep_grain_8bpc(const Dav1dGpuFilmGrainData *d, int layout, int bdmax, int16_t *grain, uint8_t *scaling);
int oracle_prep_grain_16bpc(const Dav1dGpuFilmGrainData *d, int layout, int bdmax, int16_t *grain, uint8_t *scaling);
int oracle_apply_grain_8bpc(const Dav1dGpuFilmGrainBatch *b);
int oracle_apply_grain_16bpc(const Dav1dGpuFilmGrainBatch *b);
void oracle_cdef_dsp_init_8bpc(Dav1dCdefDSPContext_8bpc *c);
void oracle_cdef_dsp_init_16bpc(Dav1dCdefDSPContext_16bpc *c);
int oracle_cdef_frame_8bpc(const Dav1dGpuCdefFrame *f, int sb128);
int oracle_cdef_frame_16bpc(const Dav1dGpuCdefFrame *f, int sb128);
void oracle_loop_filter_dsp_init_8bpc(Dav1dLoopFilterDSPContext_8bpc *c);
void oracle_loop_filter_dsp_init_16bpc(Dav1dLoopFilterDSPContext_16bpc *c);
int oracle_loopfilter_frame_8bpc(const Dav1dGpuLoopFilterFrame *f, int sb128);
int oracle_loopfilter_frame_16bpc(const Dav1dGpuLoopFilterFrame *f, int sb128);
void oracle_loop_restoration_dsp_init_8bpc(Dav1dLoopRestorationDSPContext_8bpc *c, int bpc);
void oracle_loop_restoration_dsp_init_16bpc(Dav1dLoopRestorationDSPContext_16bpc *c, int bpc);
int oracle_lr_frame_8bpc(const Dav1dGpuLrFrame *f);
int oracle_lr_frame_16bpc(const Dav1dGpuLrFrame *f);
#endif
