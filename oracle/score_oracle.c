/*
 * score_oracle.c -- CPU restatement of the score-only alignment modes of BASELINE configs[4]
 * (SURVEY.md 8(a) a17, 8(f)3): NW / SW with linear or affine (Gotoh H/E/F) gaps.
 *
 * TEST INFRASTRUCTURE ONLY, like nw_oracle.c: loaded by tests/, __graft_entry__.smoke() and
 * bench/tool CPU-baseline legs as the checker; the product never links or calls it.
 *
 * The reference has NO implementation of these modes (README.md:7-23 marks every AG/SW cell
 * as not implemented; --gapeCost is "Unused", cmd_parser.cpp:143), so parity is UNPINNED by
 * the reference.  This file defines the semantics; what pins it:
 *   - linear gaps are the special case go == ge == g, and global mode then IS the reference's
 *     NW-LG (UpdateScore, nwalign_cpu1_st_row.cpp:4-10): tests compare against orc_fill_full,
 *     which is pinned to the reference's known answers;
 *   - orc_score_ag_mt (tiled wavefront, OpenMP) and a plain Python restatement in the tests
 *     must agree with orc_score_ag bit for bit.
 *
 * Semantics (int32; g-costs are <= 0, go <= ge <= 0; NEG = -2^29 stands for -infinity):
 *   E[i][j] = max(E[i][j-1] + ge, H[i][j-1] + go)              gap consuming seqX letters
 *   F[i][j] = max(F[i-1][j] + ge, H[i-1][j] + go)              gap consuming seqY letters
 *   H[i][j] = max(H[i-1][j-1] + s(seqY[i], seqX[j]), E[i][j], F[i][j]  [, 0 if local])
 * so a gap of length L costs go + (L-1)*ge.  Boundaries:
 *   global: H[0][0] = 0, H[0][j] = E[0][j] = go + (j-1)*ge, H[i][0] = F[i][0] = go + (i-1)*ge,
 *           E[i][0] = F[0][j] = NEG;  score = H[R][C], end = (R, C)
 *   local:  H[0][j] = H[i][0] = 0, E/F on the boundary = NEG;  score = max over all H (the
 *           boundary zeros included), end = the first (i, j) in row-major order holding it.
 * Sequences carry the dummy element 0 (src/file_formats.cpp:43-47): adjrows = R+1.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_NEG (-(1 << 29))

static inline int32_t maxi(int32_t a, int32_t b) { return a >= b ? a : b; }

static inline int32_t hdr(int64_t k, int32_t go, int32_t ge) { return k == 0 ? 0 : (int32_t)(go + (k - 1) * ge); }

/* Row-streaming restatement: O(C) memory, any size. */
int32_t orc_score_ag(const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols, const int32_t* subst,
                     int32_t substsz, int32_t go, int32_t ge, int32_t local, int64_t* iend, int64_t* jend)
{
    const int64_t C = adjcols - 1, R = adjrows - 1;
    int32_t* H = (int32_t*)malloc((size_t)(C + 1) * sizeof(int32_t)); /* row i-1, then row i */
    int32_t* F = (int32_t*)malloc((size_t)(C + 1) * sizeof(int32_t));
    for (int64_t j = 0; j <= C; j++)
    {
        H[j] = local ? 0 : hdr(j, go, ge);
        F[j] = ORC_NEG;
    }
    int32_t best = 0;
    int64_t bi = 0, bj = 0;
    for (int64_t i = 1; i <= R; i++)
    {
        const int32_t* srow = subst + (int64_t)seqY[i] * substsz;
        int32_t diag = H[0];
        H[0] = local ? 0 : hdr(i, go, ge);
        int32_t E = ORC_NEG;
        for (int64_t j = 1; j <= C; j++)
        {
            E = maxi(E + ge, H[j - 1] + go);
            F[j] = maxi(F[j] + ge, H[j] + go);
            int32_t h = maxi(maxi(diag + srow[seqX[j]], E), F[j]);
            if (local) h = maxi(h, 0);
            diag = H[j];
            H[j] = h;
            if (local && h > best)
            {
                best = h;
                bi = i;
                bj = j;
            }
        }
    }
    int32_t score = local ? best : H[C];
    if (!local)
    {
        bi = R;
        bj = C;
    }
    free(H);
    free(F);
    if (iend) *iend = bi;
    if (jend) *jend = bj;
    return score;
}

/*
 * Tiled wavefront restatement (the shape of NwAlign_Cpu4_Mt_DiagRow, nwalign_cpu4_mt_diagrow.cpp:
 * 13-111: OpenMP over the tiles of each tile anti-diagonal, barrier per diagonal), used as the
 * CPU baseline of configs[4].  Tile boundaries live in per-tile-row / per-tile-column arrays.
 */
int32_t orc_score_ag_mt(const int32_t* seqY, int64_t adjrows, const int32_t* seqX, int64_t adjcols,
                        const int32_t* subst, int32_t substsz, int32_t go, int32_t ge, int32_t local,
                        int32_t blocksz, int32_t nthreads, int64_t* iend, int64_t* jend)
{
    const int64_t R = adjrows - 1, C = adjcols - 1, B = (blocksz > 0 && blocksz <= 1024) ? blocksz : 256;
    const int64_t tr = R > 0 ? (R + B - 1) / B : 0, tc = C > 0 ? (C + B - 1) / B : 0;
    if (tr == 0 || tc == 0) return orc_score_ag(seqY, adjrows, seqX, adjcols, subst, substsz, go, ge, local, iend, jend);
    /* row boundary b (row b*B, and row R for b == tr): H and F over columns 0..C;
       column boundary c (column c*B): H and E over rows 0..R */
    int32_t* RH = (int32_t*)malloc((size_t)(tr + 1) * (size_t)(C + 1) * sizeof(int32_t));
    int32_t* RF = (int32_t*)malloc((size_t)(tr + 1) * (size_t)(C + 1) * sizeof(int32_t));
    int32_t* CH = (int32_t*)malloc((size_t)(tc + 1) * (size_t)(R + 1) * sizeof(int32_t));
    int32_t* CE = (int32_t*)malloc((size_t)(tc + 1) * (size_t)(R + 1) * sizeof(int32_t));
    int64_t* tbest = (int64_t*)malloc((size_t)(tr * tc) * 3 * sizeof(int64_t));
    for (int64_t j = 0; j <= C; j++)
    {
        RH[j] = local ? 0 : hdr(j, go, ge);
        RF[j] = ORC_NEG;
    }
    for (int64_t i = 0; i <= R; i++)
    {
        CH[i] = local ? 0 : hdr(i, go, ge);
        CE[i] = ORC_NEG;
    }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    for (int64_t d = 0; d < tr + tc - 1; d++)
    {
        const int64_t t0 = d < tc ? 0 : d - tc + 1, t1 = d < tr ? d : tr - 1;
#pragma omp parallel for schedule(static)
        for (int64_t ti = t0; ti <= t1; ti++)
        {
            const int64_t tj = d - ti;
            const int64_t i0 = ti * B, j0 = tj * B;
            const int64_t i1 = (i0 + B < R) ? i0 + B : R, j1 = (j0 + B < C) ? j0 + B : C;
            const int64_t w = j1 - j0;
            int32_t H[1025], F[1025];  /* B <= 1024 */
            const int32_t* th = RH + ti * (C + 1) + j0;
            const int32_t* tf = RF + ti * (C + 1) + j0;
            for (int64_t c = 0; c <= w; c++)
            {
                H[c] = th[c];
                F[c] = tf[c];
            }
            int32_t best = -1;
            int64_t bi = 0, bj = 0;
            for (int64_t i = i0 + 1; i <= i1; i++)
            {
                const int32_t* srow = subst + (int64_t)seqY[i] * substsz;
                int32_t diag = H[0];
                H[0] = CH[tj * (R + 1) + i];
                int32_t E = CE[tj * (R + 1) + i];
                for (int64_t c = 1; c <= w; c++)
                {
                    E = maxi(E + ge, H[c - 1] + go);
                    F[c] = maxi(F[c] + ge, H[c] + go);
                    int32_t h = maxi(maxi(diag + srow[seqX[j0 + c]], E), F[c]);
                    if (local) h = maxi(h, 0);
                    diag = H[c];
                    H[c] = h;
                    if (local && h > best)
                    {
                        best = h;
                        bi = i;
                        bj = j0 + c;
                    }
                }
                CH[(tj + 1) * (R + 1) + i] = H[w];
                CE[(tj + 1) * (R + 1) + i] = E;
            }
            int32_t* bh = RH + (ti + 1) * (C + 1) + j0;
            int32_t* bf = RF + (ti + 1) * (C + 1) + j0;
            for (int64_t c = 1; c <= w; c++)
            {
                bh[c] = H[c];
                bf[c] = F[c];
            }
            if (tj == 0)
            {
                bh[0] = CH[i1];
                bf[0] = local ? ORC_NEG : hdr(i1, go, ge);
            }
            int64_t* tb = tbest + (ti * tc + tj) * 3;
            tb[0] = best;
            tb[1] = bi;
            tb[2] = bj;
        }
    }
    int32_t score;
    int64_t bi = R, bj = C;
    if (local)
    {
        /* max over tiles; ties -> smallest (i, j) in row-major order; 0 -> (0, 0) */
        int64_t best = 0;
        bi = 0;
        bj = 0;
        for (int64_t k = 0; k < tr * tc; k++)
        {
            const int64_t* tb = tbest + k * 3;
            if (tb[0] > best || (tb[0] == best && best > 0 && (tb[1] < bi || (tb[1] == bi && tb[2] < bj))))
            {
                best = tb[0];
                bi = tb[1];
                bj = tb[2];
            }
        }
        score = (int32_t)best;
    }
    else
        score = RH[tr * (C + 1) + C];
    free(RH);
    free(RF);
    free(CH);
    free(CE);
    free(tbest);
    if (iend) *iend = bi;
    if (jend) *jend = bj;
    return score;
}
