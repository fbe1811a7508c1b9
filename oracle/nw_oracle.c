/*
 * nw_oracle.c -- CPU restatement of the reference's NW-LG path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: it may be loaded
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and by
 * nothing else.  The product (gpuseqalign_amd) never links or calls it.
 *
 * Every function restates one function of markods/GpuSeqAlign (paths relative
 * to the reference checkout) with 64-bit indexing instead of the reference's
 * `int` indexing (src/math.hpp:5 overflows above 46340^2 cells).  Results are
 * identical to the reference wherever the reference itself is defined.
 *
 * Pinning: the reference cannot be built in this image (its CPU sources pull
 * cuda_runtime.h and link cudaMalloc/cudaFree through src/memory.hpp; there is
 * no libcudart here and stand-ins are not allowed), so this restatement is
 * pinned against the reference's own recorded outputs (SURVEY.md 8c known
 * answers, copied into tests/golden/known_answers.json) by
 * tests/test_oracle_golden.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EL(m, cols, i, j) ((m)[(int64_t)(cols) * (int64_t)(i) + (int64_t)(j)])

static inline int32_t max3i(int32_t a, int32_t b, int32_t c)
{
    int32_t m = a >= b ? a : b;
    return m >= c ? m : c;
}

/* One cell of the recurrence: src/nwalign_cpu1_st_row.cpp:4-10 (UpdateScore). */
static inline int32_t cell(int32_t diag, int32_t up, int32_t left, int32_t s, int32_t g)
{
    return max3i(diag + s, up + g, left + g);
}

/*
 * orc_fill_full -- NwAlign_Cpu1_St_Row (src/nwalign_cpu1_st_row.cpp:12-67).
 * seqY/seqX carry the dummy header element 0 (src/file_formats.cpp:43-47);
 * score is adjrows x adjcols row-major; returns align_cost (:62).
 */
int32_t orc_fill_full(const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols,
                      const int32_t* subst, int32_t substsz, int32_t g, int32_t* score)
{
    for (int64_t i = 0; i < adjrows; i++) EL(score, adjcols, i, 0) = (int32_t)(i * g); /* :39-42 */
    for (int64_t j = 0; j < adjcols; j++) EL(score, adjcols, 0, j) = (int32_t)(j * g); /* :43-46 */
    for (int64_t i = 1; i < adjrows; i++)                                              /* :54-60 */
    {
        const int32_t* srow = subst + (int64_t)seqY[i] * substsz;
        int32_t* prev = score + (i - 1) * adjcols;
        int32_t* curr = score + i * adjcols;
        for (int64_t j = 1; j < adjcols; j++)
            curr[j] = cell(prev[j - 1], prev[j], curr[j - 1], srow[seqX[j]], g);
    }
    return EL(score, adjcols, adjrows - 1, adjcols - 1);
}

/*
 * orc_fill_full_mt -- NwAlign_Cpu4_Mt_DiagRow (src/nwalign_cpu4_mt_diagrow.cpp:13-111):
 * square blocks of `blocksz`, one `omp for schedule(static)` per block anti-diagonal
 * with its implicit barrier (:79-103).  Used as the CPU timing baseline.
 */
int32_t orc_fill_full_mt(const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t g, int32_t* score,
                         int32_t blocksz, int32_t nthreads)
{
    const int64_t rows = adjrows - 1, cols = adjcols - 1;
    const int64_t rowblocks = (rows + blocksz - 1) / blocksz;
    const int64_t colblocks = (cols + blocksz - 1) / blocksz;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
#pragma omp for schedule(static) nowait
        for (int64_t i = 0; i < adjrows; i++) EL(score, adjcols, i, 0) = (int32_t)(i * g);
#pragma omp for schedule(static)
        for (int64_t j = 0; j < adjcols; j++) EL(score, adjcols, 0, j) = (int32_t)(j * g);
        for (int64_t s = 0; s < colblocks - 1 + rowblocks; s++)
        {
            int64_t tbeg = s - (colblocks - 1) > 0 ? s - (colblocks - 1) : 0;
            int64_t tend = s + 1 < rowblocks ? s + 1 : rowblocks;
#pragma omp for schedule(static)
            for (int64_t t = tbeg; t < tend; t++)
            {
                int64_t ibeg = 1 + t * blocksz, jbeg = 1 + (s - t) * blocksz;
                int64_t iend = ibeg + blocksz < 1 + rows ? ibeg + blocksz : 1 + rows;
                int64_t jend = jbeg + blocksz < 1 + cols ? jbeg + blocksz : 1 + cols;
                for (int64_t i = ibeg; i < iend; i++)
                {
                    const int32_t* srow = subst + (int64_t)seqY[i] * substsz;
                    int32_t* prev = score + (i - 1) * adjcols;
                    int32_t* curr = score + i * adjcols;
                    for (int64_t j = jbeg; j < jend; j++)
                        curr[j] = cell(prev[j - 1], prev[j], curr[j - 1], srow[seqX[j]], g);
                }
            }
        }
    }
    return EL(score, adjcols, adjrows - 1, adjcols - 1);
}

/* djb2-xor step used by every reference hash (src/nwtrace1_plain.cpp:118-127, :134-151). */
static inline uint32_t djb2x(uint32_t h, uint32_t v) { return ((h << 5) + h) ^ v; }

/* orc_hash_full -- NwHash1_Plain (src/nwtrace1_plain.cpp:133-154). */
uint32_t orc_hash_full(const int32_t* score, int64_t adjrows, int64_t adjcols)
{
    uint32_t h = 5381;
    const int64_t n = adjrows * adjcols;
    for (int64_t k = 0; k < n; k++) h = djb2x(h, (uint32_t)score[k]);
    return h;
}

/*
 * Run-length edit-trace builder shared by Trace1/Trace2: the reference walks from
 * the bottom-right corner, pushes (prev_edit, reversed count digits) when the edit
 * letter changes and reverses the whole string at the end
 * (src/nwtrace1_plain.cpp:81-106, src/nwtrace2_sparse.cpp:216-238).
 */
typedef struct
{
    char* buf;
    int64_t cap, len;
    int64_t same;
    char prev;
    int overflow;
} rle_t;

static void rle_push(rle_t* r, char edit)
{
    if (edit != r->prev && r->prev != '\0')
    {
        char digits[24];
        int nd = 0;
        int64_t c = r->same;
        do { digits[nd++] = (char)('0' + (c % 10)); c /= 10; } while (c);
        /* reference appends the reversed decimal string, then reverses everything */
        if (r->len + 1 + nd > r->cap) { r->overflow = 1; }
        else
        {
            r->buf[r->len++] = r->prev;
            for (int k = 0; k < nd; k++) r->buf[r->len++] = digits[k];
        }
        r->same = 1;
    }
    else if (edit == r->prev)
        r->same++;
    r->prev = edit;
}

static uint32_t rle_finish(rle_t* r)
{
    for (int64_t a = 0, b = r->len - 1; a < b; a++, b--)
    {
        char t = r->buf[a];
        r->buf[a] = r->buf[b];
        r->buf[b] = t;
    }
    uint32_t h = 5381;
    for (int64_t k = 0; k < r->len; k++) h = djb2x(h, (uint32_t)(int32_t)r->buf[k]);
    if (r->len < r->cap) r->buf[r->len] = '\0';
    return h;
}

/*
 * orc_trace_full -- NwTrace1_Plain (src/nwtrace1_plain.cpp:6-131) without the debug
 * trace.  Tie-break: diagonal by default when i>0 && j>0, then up if strictly greater,
 * then left if strictly greater (:46-77).  Returns trace_hash; the edit string
 * ("12=3X1D" style) goes to `edit` (NUL-terminated when room).  Returns 0 and sets
 * *edit_len = -1 when the buffer is too small.
 */
uint32_t orc_trace_full(const int32_t* score, const int32_t* seqY, int64_t adjrows,
                        const int32_t* seqX, int64_t adjcols, char* edit, int64_t cap, int64_t* edit_len)
{
    rle_t r = {edit, cap, 0, 1, '\0', 0};
    int64_t i = adjrows - 1, j = adjcols - 1;
    for (;;)
    {
        int64_t mx = INT64_MIN;
        int di = 0, dj = 0;
        char e = '\0';
        if (i > 0 && j > 0)
        {
            mx = EL(score, adjcols, i - 1, j - 1);
            di = -1; dj = -1;
            e = (seqX[j] == seqY[i]) ? '=' : 'X';
        }
        if (i > 0 && mx < EL(score, adjcols, i - 1, j))
        {
            mx = EL(score, adjcols, i - 1, j);
            di = -1; dj = 0; e = 'I';
        }
        if (j > 0 && mx < EL(score, adjcols, i, j - 1))
        {
            mx = EL(score, adjcols, i, j - 1);
            di = 0; dj = -1; e = 'D';
        }
        i += di;
        j += dj;
        rle_push(&r, e);
        if (di == 0 && dj == 0) break;
    }
    if (r.overflow) { *edit_len = -1; return 0; }
    uint32_t h = rle_finish(&r);
    *edit_len = r.len;
    return h;
}

/* Letter used for the padded region of the sparse (mlsp) matrix: the reference
 * zero-fills the padded tail of seqX_gpu/seqY_gpu (nwalign_gpu9_mlsp_diagdiagdiag.cu:469-478). */
static inline int32_t padded_letter(const int32_t* seq, int64_t adjlen, int64_t k)
{
    return k < adjlen ? seq[k] : 0;
}

/*
 * orc_sparse_headers -- the tile-header (mlsp) representation that the reference's
 * gpu7/gpu8/gpu9 kernels leave in tileHrowMat/tileHcolMat for tile geometry
 * (tBy rows x tBx cols): Kernel A (nwalign_gpu9_mlsp_diagdiagdiag.cu:15-63) writes row 0
 * (j*g) and column 0 (i*g); Kernel B (:69-360) writes tile (i,j)'s last row into the
 * header row of tile (i+1,j) (:319-338) and its last column into the header column of
 * tile (i,j+1) (:340-358), with the corner rule at :208-217.  Equivalently: every
 * header element is the value of the padded score matrix (padding letter 0) at its
 * position.  Padded sizes follow the host code (:416-431).
 * hrow: trows*tcols*(1+tBx) ints, hcol: trows*tcols*(1+tBy) ints.
 * Rows are streamed (two rows of Cp+1 ints), so any size fits in memory.
 * Returns align_cost = H[adjrows-1][adjcols-1].
 */
int32_t orc_sparse_headers(const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols,
                           const int32_t* subst, int32_t substsz, int32_t g, int32_t tBy, int32_t tBx,
                           int32_t* hrow, int32_t* hcol)
{
    int64_t trows = (adjrows - 1 + tBy - 1) / tBy, tcols = (adjcols - 1 + tBx - 1) / tBx;
    if (trows < 1) trows = 1;
    if (tcols < 1) tcols = 1;
    const int64_t Rp = trows * tBy, Cp = tcols * tBx;
    int32_t* prev = (int32_t*)malloc((size_t)(Cp + 1) * sizeof(int32_t));
    int32_t* curr = (int32_t*)malloc((size_t)(Cp + 1) * sizeof(int32_t));
    int32_t* xl = (int32_t*)malloc((size_t)(Cp + 1) * sizeof(int32_t));
    for (int64_t j = 0; j <= Cp; j++) xl[j] = padded_letter(seqX, adjcols, j);
    int32_t cost = 0;
    for (int64_t i = 0; i <= Rp; i++)
    {
        if (i == 0)
            for (int64_t j = 0; j <= Cp; j++) curr[j] = (int32_t)(j * g);
        else
        {
            const int32_t* srow = subst + (int64_t)padded_letter(seqY, adjrows, i) * substsz;
            curr[0] = (int32_t)(i * g);
            for (int64_t j = 1; j <= Cp; j++) curr[j] = cell(prev[j - 1], prev[j], curr[j - 1], srow[xl[j]], g);
        }
        if (i == adjrows - 1) cost = curr[adjcols - 1];
        /* header row of tile row iT = i / tBy */
        if (i % tBy == 0 && i / tBy < trows)
        {
            int64_t iT = i / tBy;
            for (int64_t jT = 0; jT < tcols; jT++)
                memcpy(hrow + (iT * tcols + jT) * (1 + tBx), curr + jT * tBx, (size_t)(1 + tBx) * sizeof(int32_t));
        }
        /* header column element (i - iT*tBy) of every tile row iT whose span [iT*tBy, iT*tBy+tBy] holds i */
        for (int64_t iT = (i / tBy) - (i % tBy == 0 && i > 0 ? 1 : 0); iT <= i / tBy && iT < trows; iT++)
        {
            if (iT < 0) continue;
            int64_t e = i - iT * tBy;
            for (int64_t jT = 0; jT < tcols; jT++) hcol[(iT * tcols + jT) * (1 + tBy) + e] = curr[jT * tBx];
        }
        int32_t* t = prev;
        prev = curr;
        curr = t;
    }
    free(prev);
    free(curr);
    free(xl);
    return cost;
}

/*
 * orc_hash_stream -- score_hash + align_cost of the full matrix without storing it.
 * This is what NwHash2_Sparse (src/nwtrace2_sparse.cpp:263-340) computes in practice:
 * it calls NwTrace2_GetTileAndElemIJ with the constant (adjrows-1, adjcols-1) (:293), so
 * after saturation neither header branch fires and the hash is a row-streaming
 * recompute equal to NwHash1_Plain.
 */
uint32_t orc_hash_stream(const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols,
                         const int32_t* subst, int32_t substsz, int32_t g, int32_t* align_cost)
{
    int32_t* prev = (int32_t*)malloc((size_t)adjcols * sizeof(int32_t));
    int32_t* curr = (int32_t*)malloc((size_t)adjcols * sizeof(int32_t));
    uint32_t h = 5381;
    for (int64_t i = 0; i < adjrows; i++)
    {
        if (i == 0)
            for (int64_t j = 0; j < adjcols; j++) curr[j] = (int32_t)(j * g);
        else
        {
            const int32_t* srow = subst + (int64_t)seqY[i] * substsz;
            curr[0] = (int32_t)(i * g);
            for (int64_t j = 1; j < adjcols; j++) curr[j] = cell(prev[j - 1], prev[j], curr[j - 1], srow[seqX[j]], g);
        }
        for (int64_t j = 0; j < adjcols; j++) h = djb2x(h, (uint32_t)curr[j]);
        int32_t* t = prev;
        prev = curr;
        curr = t;
    }
    if (align_cost) *align_cost = prev[adjcols - 1];
    free(prev);
    free(curr);
    return h;
}

/* ---- Trace2 (sparse) restatement ------------------------------------------------ */

typedef struct
{
    int64_t iTile, jTile, iTileElem, jTileElem;
} tij_t;

typedef struct
{
    const int32_t *hrow, *hcol, *seqY, *seqX, *subst;
    int64_t adjrows, adjcols, tileHdrMatRows, tileHdrMatCols, tileHrowLen, tileHcolLen;
    int32_t substsz, g;
} sparse_t;

/* NwTrace2_GetTileAndElemIJ (src/nwtrace2_sparse.cpp:8-38), saturation included. */
static void get_tile_and_elem(const sparse_t* s, int64_t i, int64_t j, tij_t* co)
{
    co->iTile = i / (s->tileHcolLen - 1);
    co->jTile = j / (s->tileHrowLen - 1);
    co->iTileElem = i % (s->tileHcolLen - 1);
    co->jTileElem = j % (s->tileHrowLen - 1);
    if (co->iTile == s->tileHdrMatRows) { co->iTile -= 1; co->iTileElem += s->tileHcolLen - 1; }
    if (co->jTile == s->tileHdrMatCols) { co->jTile -= 1; co->jTileElem += s->tileHrowLen - 1; }
}

/* NwTrace2_AlignTile (src/nwtrace2_sparse.cpp:40-96): recompute one tile from its headers,
 * up to the current element, writing 0 for artificial elements (:82-87). */
static void align_tile(const sparse_t* s, int32_t* tile, const tij_t* co)
{
    const int64_t W = s->tileHrowLen, Hh = s->tileHcolLen;
    const int64_t k = s->tileHdrMatCols * co->iTile + co->jTile;
    for (int64_t j = 0; j < W; j++) tile[j] = s->hrow[k * W + j];
    for (int64_t i = 0; i < Hh; i++) tile[i * W] = s->hcol[k * Hh + i];
    const int64_t ibeg = co->iTile * (Hh - 1), jbeg = co->jTile * (W - 1);
    const int64_t iend = Hh < co->iTileElem + 1 ? Hh : co->iTileElem + 1;
    const int64_t jend = W < co->jTileElem + 1 ? W : co->jTileElem + 1;
    for (int64_t i = 1; i < iend; i++)
        for (int64_t j = 1; j < jend; j++)
        {
            if (ibeg + i >= s->adjrows || jbeg + j >= s->adjcols) { tile[i * W + j] = 0; continue; }
            int32_t sc = s->subst[(int64_t)s->seqY[ibeg + i] * s->substsz + s->seqX[jbeg + j]];
            tile[i * W + j] = cell(tile[(i - 1) * W + j - 1], tile[(i - 1) * W + j], tile[i * W + j - 1], sc, s->g);
        }
}

/*
 * orc_trace_sparse -- NwTrace2_Sparse (src/nwtrace2_sparse.cpp:102-257) without the
 * debug trace; also returns the align_cost the mlsp `align` computes by recomputing the
 * last tile (nwalign_gpu9_mlsp_diagdiagdiag.cu:713-716).
 */
uint32_t orc_trace_sparse(const int32_t* hrow, const int32_t* hcol, int64_t trows, int64_t tcols,
                          int64_t tileHrowLen, int64_t tileHcolLen,
                          const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols,
                          const int32_t* subst, int32_t substsz, int32_t g,
                          char* edit, int64_t cap, int64_t* edit_len, int32_t* align_cost)
{
    sparse_t s = {hrow, hcol, seqY, seqX, subst, adjrows, adjcols, trows, tcols, tileHrowLen, tileHcolLen, substsz, g};
    const int64_t W = tileHrowLen;
    int32_t* tile = (int32_t*)calloc((size_t)(tileHrowLen * tileHcolLen), sizeof(int32_t));
    int64_t i = adjrows - 1, j = adjcols - 1;
    tij_t co;
    get_tile_and_elem(&s, i, j, &co);
    align_tile(&s, tile, &co);
    if (align_cost) *align_cost = tile[co.iTileElem * W + co.jTileElem];
    rle_t r = {edit, cap, 0, 1, '\0', 0};
    for (;;)
    {
        int64_t mx = INT64_MIN;
        int di = 0, dj = 0;
        char e = '\0';
        if (co.iTileElem > 0 && co.jTileElem > 0)
        {
            mx = tile[(co.iTileElem - 1) * W + co.jTileElem - 1];
            di = -1; dj = -1;
            e = (seqX[j] == seqY[i]) ? '=' : 'X';
        }
        if (co.iTileElem > 0 && mx < tile[(co.iTileElem - 1) * W + co.jTileElem])
        {
            mx = tile[(co.iTileElem - 1) * W + co.jTileElem];
            di = -1; dj = 0; e = 'I';
        }
        if (co.jTileElem > 0 && mx < tile[co.iTileElem * W + co.jTileElem - 1])
        {
            mx = tile[co.iTileElem * W + co.jTileElem - 1];
            di = 0; dj = -1; e = 'D';
        }
        i += di;
        j += dj;
        co.iTileElem += di;
        co.jTileElem += dj;
        int64_t diT = -(co.iTileElem == 0 && co.iTile > 0);
        int64_t djT = -(co.jTileElem == 0 && co.jTile > 0);
        if (diT != 0 || djT != 0)
        {
            co.iTile += diT;
            co.jTile += djT;
            if (co.iTileElem == 0 && di != 0) co.iTileElem = tileHcolLen - 1;
            if (co.jTileElem == 0 && dj != 0) co.jTileElem = tileHrowLen - 1;
            align_tile(&s, tile, &co);
        }
        rle_push(&r, e);
        if (di == 0 && dj == 0) break;
    }
    free(tile);
    if (r.overflow) { *edit_len = -1; return 0; }
    uint32_t h = rle_finish(&r);
    *edit_len = r.len;
    return h;
}

/* orc_version -- lets the loader check it got the intended build. */
int32_t orc_version(void) { return 1; }
