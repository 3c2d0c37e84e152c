// Issue-rate microbenchmark (tools only; not part of the library): SALU / VALU / mixed streams of
// independent instructions on 8 waves per SIMD, to find which issue port binds an instruction mix.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 4096
template <int NS, int NV>
__global__ __launch_bounds__(1024) void k(unsigned* out, unsigned seed) {
    unsigned s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3, s4 = seed + 4, s5 = seed + 5, s6 = seed + 6, s7 = seed + 7;
    unsigned v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (NS == 8 && NV == 0)
                asm volatile("s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 3\n s_add_u32 %2, %2, 3\n s_add_u32 %3, %3, 3\n"
                             "s_add_u32 %4, %4, 3\n s_add_u32 %5, %5, 3\n s_add_u32 %6, %6, 3\n s_add_u32 %7, %7, 3"
                             : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7) : : "scc");
            if (NV == 8 && NS == 0)
                asm volatile("v_add_u32 %0, %0, 3\n v_add_u32 %1, %1, 3\n v_add_u32 %2, %2, 3\n v_add_u32 %3, %3, 3\n"
                             "v_add_u32 %4, %4, 3\n v_add_u32 %5, %5, 3\n v_add_u32 %6, %6, 3\n v_add_u32 %7, %7, 3"
                             : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
            if (NV == 8 && NS == 8)
                asm volatile("s_add_u32 %0, %0, 3\n v_add_u32 %8, %8, 3\n s_add_u32 %1, %1, 3\n v_add_u32 %9, %9, 3\n"
                             "s_add_u32 %2, %2, 3\n v_add_u32 %10, %10, 3\n s_add_u32 %3, %3, 3\n v_add_u32 %11, %11, 3\n"
                             "s_add_u32 %4, %4, 3\n v_add_u32 %12, %12, 3\n s_add_u32 %5, %5, 3\n v_add_u32 %13, %13, 3\n"
                             "s_add_u32 %6, %6, 3\n v_add_u32 %14, %14, 3\n s_add_u32 %7, %7, 3\n v_add_u32 %15, %15, 3"
                             : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7),
                               "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : : "scc");
            if (NV == 8 && NS == 4)
                asm volatile("s_add_u32 %0, %0, 3\n v_add_u32 %4, %4, 3\n v_add_u32 %5, %5, 3\n s_add_u32 %1, %1, 3\n"
                             "v_add_u32 %6, %6, 3\n v_add_u32 %7, %7, 3\n s_add_u32 %2, %2, 3\n v_add_u32 %8, %8, 3\n"
                             "v_add_u32 %9, %9, 3\n s_add_u32 %3, %3, 3\n v_add_u32 %10, %10, 3\n v_add_u32 %11, %11, 3"
                             : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3),
                               "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : : "scc");
        }
    }
    unsigned r = s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7 ^ v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;  // vector store
}
template <int NS, int NV>
void run(unsigned* d, int wgs, int threads, const char* name) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<NS, NV><<<wgs, threads>>>(d, 1);
    hipEventRecord(a);
    k<NS, NV><<<wgs, threads>>>(d, 1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess || hipGetLastError() != hipSuccess) printf("%s: error %s\n", name, hipGetErrorString(e));
    float ms; hipEventElapsedTime(&ms, a, b);
    const double waves_per_simd = (double)wgs * threads / 64 / (256 * 4);
    const double per_wave = (double)ITERS * 4;  // instructions of each kind per wave
    const double cyc = ms * 1e-3 * 2.4e9;
    printf("%-10s waves/SIMD %.0f: %.3f ms; SALU/SIMD/cyc %.3f VALU/SIMD/cyc %.3f\n", name, waves_per_simd, ms,
           NS * per_wave * waves_per_simd / cyc, NV * per_wave * waves_per_simd / cyc);
}
int main() {
    unsigned* d; hipMalloc(&d, 512 * 1024 * 4);
    for (int w : {1, 2, 4, 8}) {
        const int wgs = 256 * w / 4 * 4 / 4;  // w waves/SIMD: 4w waves per CU; 1024-thread WGs hold 16 waves
        (void)wgs;
        const int threads = 64 * 4 * w <= 1024 ? 64 * 4 * w : 1024;
        const int nwg = 256 * (64 * 4 * w) / threads;
        run<8, 0>(d, nwg, threads, "salu8");
        run<0, 8>(d, nwg, threads, "valu8");
        run<8, 8>(d, nwg, threads, "mix8+8");
        run<4, 8>(d, nwg, threads, "mix4+8");
    }
    return 0;
}
