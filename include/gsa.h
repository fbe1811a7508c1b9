/*
 * gsa.h -- C ABI of the MI355X NW-LG engine (libgsa.so).
 *
 * This is the drop-in boundary for the reference's align slot
 *     using NwAlignFn = NwStat (*)(const NwAlgParams&, NwAlgInput&, NwAlgResult&);
 * (markods/GpuSeqAlign src/nw_algorithm.hpp:11, registered in src/nw_algorithm.cpp:48-66)
 * and for the consumers the registry pairs with it (NwTrace1_Plain / NwHash1_Plain,
 * NwTrace2_Sparse / NwHash2_Sparse, src/nw_fns.hpp:22-39).  Plain pointers and sizes only.
 *
 * Conventions (identical to NwAlgInput, src/run_types.hpp:70-110):
 *  - seqY / seqX are int32 letter indices WITH the dummy header element 0
 *    (src/file_formats.cpp:43-47); adjrows = |seqY|+1, adjcols = |seqX|+1.
 *  - subst is substsz*substsz int32, row = seqY letter, column = seqX letter
 *    (src/nwalign_cpu1_st_row.cpp:6).
 *  - gapo is the linear gap cost (reference default -11, src/cmd_parser.cpp:298).
 *  - full score matrix: adjrows*adjcols int32 row-major, unpadded (nw.score).
 *  - sparse (mlsp) matrices: tileHrowMat[trows*tcols*(1+tileBx)] and
 *    tileHcolMat[trows*tcols*(1+tileBy)], tile-major row-major k = tcols*iTile + jTile
 *    (nwalign_gpu9_mlsp_diagdiagdiag.cu:15-63, :147-171, :319-358).
 *  - every int-returning function returns an NwStat code (src/run_types.hpp:12-24); the
 *    raw hipError_t of the failing runtime call is kept in the context
 *    (gsa_last_hip_error), like NwAlgResult::cudaStat.
 */
#ifndef GSA_H
#define GSA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* NwStat (src/run_types.hpp:12-24), same numbering. */
enum gsa_stat
{
    GSA_SUCCESS = 0,
    GSA_HELP_MENU_REQUESTED = 1,
    GSA_ERROR_CUDA_GENERAL = 2, /* errorCudaGeneral: HIP runtime failure */
    GSA_ERROR_MEMORY_ALLOCATION = 3,
    GSA_ERROR_MEMORY_TRANSFER = 4,
    GSA_ERROR_KERNEL_FAILURE = 5,
    GSA_ERROR_IO_STREAM = 6,
    GSA_ERROR_INVALID_FORMAT = 7,
    GSA_ERROR_INVALID_VALUE = 8,
    GSA_ERROR_INVALID_RESULT = 9
};

typedef struct gsa_ctx gsa_ctx;

/* Sparse geometry produced by a fill (NwAlgInput tileHdrMatRows/Cols, tileHrowLen/HcolLen,
 * src/run_types.hpp:97-100; set at nwalign_gpu9_mlsp_diagdiagdiag.cu:696-699). */
typedef struct gsa_sparse_geom
{
    int32_t tileBx, tileBy;
    int32_t tileHdrMatRows, tileHdrMatCols; /* trows, tcols */
    int32_t tileHrowLen, tileHcolLen;       /* 1+tileBx, 1+tileBy */
    int64_t hrowElems, hcolElems;           /* trows*tcols*(1+tileBx), trows*tcols*(1+tileBy) */
} gsa_sparse_geom;

/* Stopwatch laps of NwAlgResult::sw_align, in ms (src/stopwatch.cpp:43-50; names at
 * src/file_formats.cpp:505-519).  calc_kernel_ms is the hipEvent time of the fill kernels. */
typedef struct gsa_laps
{
    float alloc, cpy_dev, init_hdr, calc, cpy_host;
    float calc_kernel_ms;
} gsa_laps;

/* Phase-boundary callback of the host-buffer entry points (gsa_align_full, gsa_align_sparse,
 * gsa_align_sparse_pt, gsa_score): called with "align.alloc", "align.cpy_dev", "align.init_hdr",
 * "align.calc", "align.cpy_host" (and "align.calc" again after the last-tile recompute of the
 * sparse forms) at the points where the reference's align functions call Stopwatch::lap
 * (nwalign_gpu9_mlsp_diagdiagdiag.cu:435-719, nwalign_gpu3_ml_diagdiag.cu:329-593;
 * src/stopwatch.hpp:19), so an adapter drives the reference's own stopwatch:
 *     static void onLap(void* sw, const char* name) { ((Stopwatch*)sw)->lap(name); }
 *     res.sw_align.start(); gsa_set_lap_callback(ctx, onLap, &res.sw_align);
 * Called on the calling thread, before the entry point returns.  fn = NULL removes it. */
typedef void (*gsa_lap_fn)(void* user, const char* lap_name);

/* ---- context --------------------------------------------------------------------- */
/* One context per device and host thread (the reference's initNwInput, src/benchmark.cpp:175-223). */
int gsa_ctx_create(int device, gsa_ctx** out);
void gsa_ctx_destroy(gsa_ctx* ctx);
int gsa_last_hip_error(const gsa_ctx* ctx);
int gsa_device_cu_count(const gsa_ctx* ctx);
const char* gsa_version(void);
int gsa_set_lap_callback(gsa_ctx* ctx, gsa_lap_fn fn, void* user);
/* Not part of the reference's interface: the measurement / test switches, named as environment
 * variables (GSA_FULL_KERNEL, GSA_KROW_NS, ...; DESIGN.md lists them).  A context takes them from
 * the environment once, in gsa_ctx_create; this sets one for this context (value NULL: unset, the
 * built-in choice).  errorInvalidValue for a name the library does not know. */
int gsa_set_knob(gsa_ctx* ctx, const char* name, const char* value);

/* Tile height (tileBy) of the sparse representation this build produces: 1024, the rows of one
 * K-rows workgroup ticket (4 strip waves x 64 lanes x 4 rows per lane). */
int32_t gsa_sparse_tile_by(void);
/* Geometry for (adjrows, adjcols, tileBx); tileBx must be a multiple of 16 and >= 64. */
int gsa_sparse_geometry(int32_t adjrows, int32_t adjcols, int32_t tileBx, gsa_sparse_geom* geom);

/* ---- hot path, device-resident buffers (inputs already in HBM) --------------------- */
/* Enqueue the fill on `stream` (a hipStream_t; NULL = the HIP null stream); asynchronous.  Call
 * gsa_sync() before reading outputs: it also reports hand-off time-outs.  The context's error word
 * is STICKY: a time-out in any launch enqueued since the last gsa_sync() makes that gsa_sync()
 * return GSA_ERROR_KERNEL_FAILURE (launches enqueued behind the failed one give up at once), and
 * gsa_sync() then clears it, so the context is usable again.  One stream per context at a time
 * (the launches share the context's ticket word). */
int gsa_fill_full_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                      const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score, void* stream);
int gsa_fill_sparse_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                        const int32_t* subst, int32_t substsz, int32_t gapo, int32_t tileBx, int32_t* tileHrowMat,
                        int32_t* tileHcolMat, void* stream);
int gsa_sync(gsa_ctx* ctx, void* stream);

/* Pitched device layout of a full matrix.  The reference keeps its device score matrix padded
 * and crops it on the way back (nwalign_gpu3_ml_diagdiag.cu:315-325, cudaMemcpy2D at :585-588,
 * src/memory.hpp:217); these entry points take the row pitch `ld` (>= adjcols, in ints) of such a
 * device matrix: cell (i, j) at score[i*ld + j].  Every ld >= adjcols gives the same values.
 * gsa_full_pitch(adjcols) is the pitch this engine writes fastest: ld = 1 (mod 32), and with the
 * matrix placed gsa_full_base_offset() ints past a 128-byte boundary (cell (1, 0) on one), all
 * cells of an anti-diagonal share their offset within a 128-byte line, so the wavefront's row
 * segments are stored as whole aligned lines (no partial-line writes). */
int32_t gsa_full_pitch(int32_t adjcols);
int32_t gsa_full_base_offset(void);
int gsa_fill_full_pitched_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX,
                              int32_t adjcols, const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score,
                              int32_t ld, void* stream);
/* Peak resource use of the fills launched on this context since its creation or the last reset:
 * the reference's NwAlgResult peak-alloc columns (updateNwAlgPeakMemUsage, nwalign_shared.cpp:5-25).
 * shmem/locmem/regmem = per-workgroup LDS, per-lane scratch x threads, per-lane VGPRs x 4 B x
 * threads, each times the workgroups resident at once; glmem = device bytes the context holds
 * (scratch and hand-off buffers, plus the host-buffer entry points' input/output copies). */
typedef struct gsa_mem_stats
{
    int64_t glmem_peak_allocs, shmem_peak_allocs, locmem_peak_allocs, regmem_peak_allocs;
} gsa_mem_stats;
int gsa_mem_stats_get(const gsa_ctx* ctx, gsa_mem_stats* out);
int gsa_mem_stats_reset(gsa_ctx* ctx);
/* Hand-off watchdog: a wait inside a fill that sees no progress for this long gives up and sets
 * the error word (default 1 s; 0 = give up at the first unmet poll, for tests of the error path).
 * Applies to launches enqueued after the call. */
int gsa_set_watchdog(gsa_ctx* ctx, int64_t microseconds);

/* ---- batched fills: many independent pairs in ONE persistent launch ------------------- */
/* Device pointers of one pair: score for full fills (adjrows*adjcols), the two header
 * matrices for sparse fills (sizes from gsa_sparse_geometry). */
typedef struct gsa_pair_dev
{
    const int32_t* seqY;
    int32_t adjrows;
    const int32_t* seqX;
    int32_t adjcols;
    int32_t* score;
    int32_t* tileHrowMat;
    int32_t* tileHcolMat;
} gsa_pair_dev;
/* `pairs` is a host array of `npairs` entries; results are identical to one fill per pair.
 * The reference runs pairs one at a time through its benchmark loop (src/benchmark.cpp:
 * 393-520); a batch replaces that loop for throughput runs (BASELINE configs[3]).
 * Launches on one context must be ordered (same stream, or synchronised).  Asynchronous: a full
 * batch times its candidate schedules on its first launches with HIP events that are read only
 * once complete (never a host wait); the host blocks only when more than 4 launches' descriptors
 * are in flight on the context. */
int gsa_fill_full_batch_dev(gsa_ctx* ctx, int32_t npairs, const gsa_pair_dev* pairs, const int32_t* subst,
                            int32_t substsz, int32_t gapo, void* stream);
/* As gsa_fill_full_batch_dev, pair p's matrix with row pitch lds[p] (>= its adjcols; see
 * gsa_full_pitch). */
int gsa_fill_full_batch_pitched_dev(gsa_ctx* ctx, int32_t npairs, const gsa_pair_dev* pairs, const int32_t* lds,
                                    const int32_t* subst, int32_t substsz, int32_t gapo, void* stream);
int gsa_fill_sparse_batch_dev(gsa_ctx* ctx, int32_t npairs, const gsa_pair_dev* pairs, const int32_t* subst,
                              int32_t substsz, int32_t gapo, int32_t tileBx, void* stream);

/* ---- NwAlignFn equivalents, host buffers (alloc + H2D + fill + D2H, laps as the
 * reference's NwAlign_Gpu3_Ml_DiagDiag / NwAlign_Gpu9_Mlsp_DiagDiagDiag) -------------- */
int gsa_align_full(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                   const int32_t* subst, int32_t substsz, int32_t gapo, int32_t* score_out, int32_t* align_cost,
                   gsa_laps* laps);
int gsa_align_sparse(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                     const int32_t* subst, int32_t substsz, int32_t gapo, int32_t tileBx, int32_t* tileHrowMat_out,
                     int32_t* tileHcolMat_out, gsa_sparse_geom* geom, int32_t* align_cost, gsa_laps* laps);

/* mlsppt ("multi-launch sparse with parallel transfer", named in the reference's README.md:39,
 * never implemented there): as gsa_align_sparse, but the header matrices are copied back to
 * the host tile row by tile row WHILE the fill runs (the kernel flags each finished
 * super-strip in host-mapped memory).  Same outputs; the laps' cpy_host is only the tail
 * copied after the fill ends. */
int gsa_align_sparse_pt(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                        const int32_t* subst, int32_t substsz, int32_t gapo, int32_t tileBx, int32_t* tileHrowMat_out,
                        int32_t* tileHcolMat_out, gsa_sparse_geom* geom, int32_t* align_cost, gsa_laps* laps);

/* Measurement aid, not part of the reference's interface: with GSA_STAMPS=1 in the environment a
 * fused full fill records stamps: [start, end] (s_memrealtime, 100 MHz) and [start,
 * end] (s_memtime, shader clock) per pass-1 strip, then [claimed, ready, done] (s_memrealtime) per
 * expansion task; a K-rows sparse fill or a full fill's separate pass 1 records its strip ledger:
 * [realtime start, end, shader clock start, end, cycles waiting for input, waits, four block spans of
 * a diagnostic build] per strip (10 words).  Copies
 * the last such launch's *n stamps
 * into out (cap >= *n, else errorInvalidValue; out may be null to query *n); synchronizes the stream
 * that launch ran on. */
int gsa_debug_stamps(gsa_ctx* ctx, uint64_t* out, int64_t cap, int64_t* n);

/* Measurement aid, not part of the reference's interface: with timing on, every two-pass full fill
 * (gsa_fill_full*_dev) records HIP events before pass 1, between the passes and
 * after pass 2 on its stream, and pass 2's workgroups record their shader cycles (s_memtime) and
 * 100 MHz ticks (s_memrealtime) from start to end.  gsa_last_full_timing waits for the last such
 * fill and returns the pass times and the effective shader clock over pass 2's workgroups (median
 * and cycle-weighted mean), so a slow box shows as a low clock.  A fused fill (one launch) has
 * pass1_ms = -1, its whole time in pass2_ms and no clock.  A pipelined batch (groups > 0: pass 1 of
 * pair group g + 1 beside the expansion of group g) has group 0's pass 1 (alone on the chip) in
 * pass1_ms, everything after it in pass2_ms and the clock of its last expansion launch.
 * errorInvalidValue: no timed fill. */
typedef struct gsa_full_timing
{
    float pass1_ms, pass2_ms;
    float clock_ghz_median, clock_ghz_mean;
    int64_t workgroups;  /* pass-2 workgroups whose clock was resolved (>= 1 us) */
    int32_t fused;
    int32_t groups;  /* pipelined batch: pair groups (0: not pipelined) */
} gsa_full_timing;
int gsa_set_full_timing(gsa_ctx* ctx, int32_t on);
int gsa_last_full_timing(gsa_ctx* ctx, gsa_full_timing* out);

/* ---- consumers (host), the reference's L4 ----------------------------------------- */
/* NwHash1_Plain (src/nwtrace1_plain.cpp:133-154). */
uint32_t gsa_hash_full(const int32_t* score, int32_t adjrows, int32_t adjcols);
/* NwTrace1_Plain (src/nwtrace1_plain.cpp:6-131); edit string NUL-terminated if room.
 * Returns GSA_ERROR_MEMORY_ALLOCATION if `cap` is too small. */
int gsa_trace_full(const int32_t* score, const int32_t* seqY, int32_t adjrows, const int32_t* seqX,
                   int32_t adjcols, char* edit, int64_t cap, int64_t* edit_len, uint32_t* trace_hash);
/* NwTrace2_Sparse (src/nwtrace2_sparse.cpp:102-257) + the align_cost recompute of the mlsp
 * align functions (nwalign_gpu9_mlsp_diagdiagdiag.cu:713-716). */
int gsa_trace_sparse(const int32_t* tileHrowMat, const int32_t* tileHcolMat, const gsa_sparse_geom* geom,
                     const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                     const int32_t* subst, int32_t substsz, int32_t gapo, char* edit, int64_t cap,
                     int64_t* edit_len, uint32_t* trace_hash, int32_t* align_cost);
/* NwHash2_Sparse (src/nwtrace2_sparse.cpp:263-340). */
uint32_t gsa_hash_sparse(const int32_t* tileHrowMat, const int32_t* tileHcolMat, const gsa_sparse_geom* geom,
                         const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t gapo);
/* align_cost of a sparse result: NwTrace2_GetTileAndElemIJ + NwTrace2_AlignTile of the last
 * tile (nwalign_gpu9_mlsp_diagdiagdiag.cu:713-716). */
int32_t gsa_sparse_align_cost(const int32_t* tileHrowMat, const int32_t* tileHcolMat, const gsa_sparse_geom* geom,
                              const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                              const int32_t* subst, int32_t substsz, int32_t gapo);

/* ---- device-side verification ------------------------------------- */
/* The reference compares a GPU fill only through align_cost and the score / trace hashes, so
 * sparse header values off the trace path are never checked (nwtrace2_sparse.cpp:263-340).
 * These check EVERY output value against the recurrence (nwalign_cpu1_st_row.cpp:4-10) on the
 * device: a sparse result by tile consistency (each tile recomputed from its own header row
 * and column must reproduce the headers of the tiles below and to the right; row 0 / column 0
 * must be j*g / i*g; the two copies of each tile corner must agree), a full matrix cell by
 * cell against its stored neighbours.  Zero mismatches implies every value is exact.
 * Synchronous on `stream`; inputs are device pointers. */
typedef struct gsa_check_result
{
    int64_t checked;    /* values compared */
    int64_t mismatches; /* values inconsistent with the recurrence or the boundary */
    int64_t first;      /* smallest mismatching index, -1 if none: full = i*adjcols+j;
                           sparse = index into tileHrowMat, or hrowElems + index into tileHcolMat */
} gsa_check_result;
int gsa_check_sparse_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t gapo, const gsa_sparse_geom* geom,
                         const int32_t* tileHrowMat, const int32_t* tileHcolMat, gsa_check_result* out,
                         void* stream);
int gsa_check_full_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                       const int32_t* subst, int32_t substsz, int32_t gapo, const int32_t* score,
                       gsa_check_result* out, void* stream);
/* As gsa_check_full_dev for a matrix with row pitch ld (>= adjcols, gsa_fill_full_pitched_dev);
 * `first` is still i*adjcols+j. */
int gsa_check_full_pitched_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX,
                               int32_t adjcols, const int32_t* subst, int32_t substsz, int32_t gapo,
                               const int32_t* score, int32_t ld, gsa_check_result* out, void* stream);

/* The plain family's consumers over a matrix that stays in HBM (row pitch ld >= adjcols; ld =
 * adjcols for gsa_fill_full_dev output), so a 100k x 100k matrix (40 GB) is hashed and traced
 * without a host copy of it.  Results are identical to gsa_hash_full / gsa_trace_full of the
 * same matrix.  Both wait for `stream` first and are synchronous.
 * gsa_hash_full_dev: NwHash1_Plain (src/nwtrace1_plain.cpp:133-154); the hash is one serial chain
 *   over every cell, folded on the host while rows stream through two pinned buffers.
 * gsa_trace_full_dev: NwTrace1_Plain (src/nwtrace1_plain.cpp:6-131) -- the walk reads blocks of
 *   the matrix around its position; seqY/seqX are device pointers; align_cost = the last cell. */
int gsa_hash_full_dev(gsa_ctx* ctx, const int32_t* score, int32_t adjrows, int32_t adjcols, int32_t ld,
                      uint32_t* hash, void* stream);
int gsa_trace_full_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                       const int32_t* score, int32_t ld, char* edit, int64_t cap, int64_t* edit_len,
                       uint32_t* trace_hash, int32_t* align_cost, void* stream);

/* NwTrace2_Sparse (src/nwtrace2_sparse.cpp:102-257) on the device: the walk and its tile
 * recomputes run on the GPU from device-resident headers; outputs (edit string, trace hash,
 * align_cost) are identical to gsa_trace_sparse.  Synchronous on `stream`. */
int gsa_trace_sparse_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t gapo, const gsa_sparse_geom* geom,
                         const int32_t* tileHrowMat, const int32_t* tileHcolMat, char* edit, int64_t cap,
                         int64_t* edit_len, uint32_t* trace_hash, int32_t* align_cost, void* stream);

/* ---- score-only NW / SW, linear or affine gaps (BASELINE configs[4]) ---- */
/* Not in the reference (README.md:7-23 marks AG/SW unimplemented; --gapeCost is unused,
 * cmd_parser.cpp:143).  Semantics: oracle/score_oracle.c --
 *   E = max(E_left + gape, H_left + gapo), F = max(F_up + gape, H_up + gapo),
 *   H = max(H_diag + s, E, F [, 0 if local]); a gap of length L costs gapo + (L-1)*gape;
 *   global: score = H[R][C], boundaries gapo + (k-1)*gape; local: max over H, end = first
 *   cell in row-major order.  gapo == gape == g is the reference's NW-LG.  Requires
 *   gapo <= gape <= 0.  Synchronous. */
/* gsa_score_dev reads the substitution table back in stream order (it sizes the value range
 * from it) before its launch; the score kernels report errors in a control word of their own, so
 * the fills' sticky error word is left for the caller's gsa_sync.  Global scores of long pairs run
 * from both ends (the top rows forward, the bottom rows reversed, in one launch; the pair
 * transposed when only adjcols-1 suits the split); local ones too, by rows only, with a third
 * pair (the bottom rows forward from a fresh border) for the end cell and a second launch when
 * an alignment through the split row decides the result: same results, context scratch grows by
 * ~4 (adjcols + adjrows) ints and, local, by the granules of one more pass. */
typedef struct gsa_score_result
{
    int32_t score;
    int64_t i_end, j_end;  /* local: where the maximum first occurs; global: (adjrows-1, adjcols-1) */
    float calc_kernel_ms;  /* hipEvent time of the fill: for scores split in two halves (from both
                            * ends) the prep, fill and combine kernels, and a local
                            * pair's second launch when it needed one */
} gsa_score_result;
int gsa_score_dev(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
                  const int32_t* subst, int32_t substsz, int32_t gapo, int32_t gape, int32_t local,
                  gsa_score_result* out, void* stream);
/* Host buffers (alloc, copy in, fill, laps as gsa_align_*). */
int gsa_score(gsa_ctx* ctx, const int32_t* seqY, int32_t adjrows, const int32_t* seqX, int32_t adjcols,
              const int32_t* subst, int32_t substsz, int32_t gapo, int32_t gape, int32_t local,
              gsa_score_result* out, gsa_laps* laps);

#ifdef __cplusplus
}
#endif

#endif /* GSA_H */
