// lds_align_probe.hip -- does ds_read_b128 / ds_read_b64 at a 4-byte (not 16-byte) aligned LDS
// address return the 4 dwords at that address on gfx950 (unaligned LDS access mode)?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int2v __attribute__((ext_vector_type(2)));
extern __shared__ __attribute__((aligned(16))) char sm[];
__global__ void k(int* out)
{
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) ((int*)sm)[i] = i * 7 + 1;
    __syncthreads();
    const int off = lane;  // dword offset, any alignment
    int4v v;
    int2v u;
    const unsigned a = (unsigned)(size_t)(sm + 4 * off);
    asm volatile("ds_read_b128 %0, %2\n ds_read_b64 %1, %2 offset:4\n s_waitcnt lgkmcnt(0)" : "=v"(v), "=v"(u) : "v"(a) : "memory");
    int bad = 0;
    for (int j = 0; j < 4; ++j) bad |= v[j] != (off + j) * 7 + 1;
    for (int j = 0; j < 2; ++j) bad |= u[j] != (off + 1 + j) * 7 + 1;
    out[lane] = bad;
}
int main()
{
    int* d;
    (void)hipMalloc(&d, 256);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 4096, 0, d);
    int h[64];
    (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    int nb = 0;
    for (int i = 0; i < 64; ++i) nb += h[i];
    printf("misaligned ds_read_b128/b64: %d of 64 lanes wrong\n", nb);
    return 0;
}
