// nw_bidi.hip -- score-only NW from both ends: sequence reversal and the combine at the meeting row
// (nw_bidi.h).  The split is Hirschberg's / Myers-Miller's: every global path crosses from row m to
// row m + 1 once after its last cell (m, j) on row m; the forward top half gives the best prefix
// score at (m, j) in any state (H) and in the vertical-gap state (F), the reversed bottom half the
// best suffix score from (m, j) (H^r) and the one that starts with a vertical gap (F^r), and a gap
// that crosses the boundary pays its open once: score = max_j max(H + H^r, F + F^r - (go - ge)).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_bidi.h"
#include "nw_strip.h"

namespace gsa {
namespace {

__global__ void reverse_kernel(const int* src, int first, int last, int* dst)
{
    const int n = last - first + 1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gridDim.x * blockDim.x)
        dst[i] = i == 0 ? 0 : src[last + 1 - i];
}

__global__ void __launch_bounds__(1024) bidi_combine_kernel(const int* topH, const int* topF, const int* botH,
                                                            const int* botF, int m, int mb, int C, int go, int ge,
                                                            int affine, int* out)
{
    __shared__ long long red[1024];
    const long long d = (long long)go - ge;
    long long best = -(1ll << 62);
    for (int j = threadIdx.x; j <= C; j += blockDim.x)
    {
        const int jb = C - j;
        // H and F of the forward top at (m, j) and of the reversed bottom at (mb, jb), unshifted
        long long ht, ft, hb, fb;
        if (j == 0)
            ht = ft = (long long)go + (long long)(m - 1) * ge;
        else
        {
            ht = (long long)topH[kTapPad + j] - d + (long long)(m + j) * ge;
            ft = affine ? (long long)topF[kTapPad + j] + (long long)(m + j) * ge : ht;
        }
        if (jb == 0)
            hb = fb = (long long)go + (long long)(mb - 1) * ge;
        else
        {
            hb = (long long)botH[kTapPad + jb] - d + (long long)(mb + jb) * ge;
            fb = affine ? (long long)botF[kTapPad + jb] + (long long)(mb + jb) * ge : hb;
        }
        long long v = ht + hb;
        if (affine) v = max(v, ft + fb - d);
        best = max(best, v);
    }
    red[threadIdx.x] = best;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1)
    {
        if ((int)threadIdx.x < s) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = (int)red[0];
}

}  // namespace

hipError_t launch_reverse(const int* src, int first, int last, int* dst, hipStream_t stream)
{
    const int n = last - first + 2;
    const int grid = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
    hipLaunchKernelGGL(reverse_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, stream, src, first, last, dst);
    return hipGetLastError();
}

hipError_t launch_bidi_combine(const int* topH, const int* topF, const int* botH, const int* botF, int m, int mb,
                               int C, int go, int ge, bool affine, int* out, hipStream_t stream)
{
    hipLaunchKernelGGL(bidi_combine_kernel, dim3(1), dim3(1024), 0, stream, topH, topF, botH, botF, m, mb, C, go, ge,
                       affine ? 1 : 0, out);
    return hipGetLastError();
}

}  // namespace gsa
