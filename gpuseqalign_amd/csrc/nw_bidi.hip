// nw_bidi.hip -- score-only NW from both ends: sequence reversal and the combine at the meeting row
// (nw_bidi.h).  The split is Hirschberg's / Myers-Miller's: every global path crosses from row m to
// row m + 1 once after its last cell (m, j) on row m; the forward top half gives the best prefix
// score at (m, j) in any state (H) and in the vertical-gap state (F), the reversed bottom half the
// best suffix score from (m, j) (H^r) and the one that starts with a vertical gap (F^r), and a gap
// that crosses the boundary pays its open once: score = max_j max(H + H^r, F + F^r - (go - ge)).
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "nw_bidi.h"
#include "nw_strip.h"

namespace gsa {
namespace {

__global__ void __launch_bounds__(256) bidi_prep_kernel(PairDesc d0, PairDesc d1, PairDesc d2, int three, PairDesc* desc,
                                                        const int* seqY, int m, int R, const int* seqX, int C, int* ry,
                                                        int* rx, unsigned* ticket, unsigned long long* words, int* out,
                                                        const int* subst, int substsz, int* substT)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    if (t == 0)
    {
        desc[0] = d0;
        desc[1] = d1;
        if (three) desc[2] = d2;
        ticket[0] = 0;
        for (int k = 0; k < 8; ++k) words[k] = 0;
        out[0] = INT_MIN;
    }
    const int mb = R - m;
    for (int i = t; i <= mb; i += stride) ry[i] = i == 0 ? 0 : seqY[R + 1 - i];
    for (int j = t; j <= C; j += stride) rx[j] = j == 0 ? 0 : seqX[C + 1 - j];
    if (substT)
        for (int k = t; k < substsz * substsz; k += stride) substT[k] = subst[(k % substsz) * substsz + k / substsz];
}

__global__ void __launch_bounds__(256) bidi_combine_kernel(const int* topH, const int* topF, int ts, const int* botH,
                                                           const int* botF, int bs, int m, int mb, int C, int go,
                                                           int ge, int affine, int local, int* out)
{
    __shared__ int red[256];
    const long long d = (long long)go - ge;
    long long best = -(1ll << 62);
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j <= C; j += gridDim.x * blockDim.x)
    {
        const int jb = C - j;
        // H and F of the forward top at (m, j) and of the reversed bottom at (mb, jb), unshifted
        long long ht, ft, hb, fb;
        if (j == 0)
        {
            ht = ft = (long long)go + (long long)(m - 1) * ge;
            if (local)
            {
                ht = 0;
                ft = -(1ll << 40);
            }
        }
        else
        {
            ht = (long long)topH[(size_t)ts * j] - d + (long long)(m + j) * ge;
            ft = affine ? (long long)topF[(size_t)ts * j] + (long long)(m + j) * ge : ht;
        }
        if (jb == 0)
        {
            hb = fb = (long long)go + (long long)(mb - 1) * ge;
            if (local)
            {
                hb = 0;
                fb = -(1ll << 40);
            }
        }
        else
        {
            hb = (long long)botH[(size_t)bs * jb] - d + (long long)(mb + jb) * ge;
            fb = affine ? (long long)botF[(size_t)bs * jb] + (long long)(mb + jb) * ge : hb;
        }
        long long v = ht + hb;
        if (affine) v = max(v, ft + fb - d);
        best = max(best, v);
    }
    // scores stay far inside int (the fill flags anything outside int16 / 2^26)
    red[threadIdx.x] = (int)max(best, (long long)INT_MIN);
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1)
    {
        if ((int)threadIdx.x < s) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(out, red[0]);
}

__global__ void __launch_bounds__(256) bidi_seed_kernel(const unsigned long long* src, const unsigned long long* src2,
                                                        unsigned long long* dst, unsigned long long* dst2, long long n,
                                                        unsigned epoch)
{
    const unsigned long long ep = (unsigned long long)epoch << 32;
    for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < n; c += (long long)gridDim.x * blockDim.x)
    {
        dst[c] = ep | (src[c] & 0xffffffffull);
        if (dst2) dst2[c] = ep | (src2[c] & 0xffffffffull);
    }
}

}  // namespace

hipError_t launch_bidi_seed(const unsigned long long* src, const unsigned long long* src2, unsigned long long* dst,
                            unsigned long long* dst2, long long n, unsigned epoch, hipStream_t stream)
{
    const long long g = (n + 255) / 256;
    hipLaunchKernelGGL(bidi_seed_kernel, dim3(g < 256 ? (unsigned)g : 256u), dim3(256), 0, stream, src, src2, dst, dst2, n,
                       epoch);
    return hipGetLastError();
}

hipError_t launch_bidi_prep(const PairDesc& d0, const PairDesc& d1, PairDesc* desc, const int* seqY, int m, int R,
                            const int* seqX, int C, int* ry, int* rx, unsigned* ticket,
                            unsigned long long* words, int* out, const int* subst, int substsz, int* substT,
                            hipStream_t stream, const PairDesc* d2)
{
    const int n = (R - m > C ? R - m : C) + 1;
    const int grid = (n + 255) / 256 < 512 ? (n + 255) / 256 : 512;
    hipLaunchKernelGGL(bidi_prep_kernel, dim3(grid), dim3(256), 0, stream, d0, d1, d2 ? *d2 : d1, d2 ? 1 : 0, desc, seqY, m,
                       R, seqX, C, ry, rx, ticket, words, out, subst, substsz, substT);
    return hipGetLastError();
}

hipError_t launch_bidi_combine(const int* topH, const int* topF, int ts, const int* botH, const int* botF, int bs,
                               int m, int mb, int C, int go, int ge, bool affine, int* out, hipStream_t stream,
                               bool local)
{
    const int grid = (C + 1 + 255) / 256 < 256 ? (C + 1 + 255) / 256 : 256;
    hipLaunchKernelGGL(bidi_combine_kernel, dim3(grid), dim3(256), 0, stream, topH, topF, ts, botH, botF, bs, m, mb, C,
                       go, ge, affine ? 1 : 0, local ? 1 : 0, out);
    return hipGetLastError();
}

}  // namespace gsa
