// valu_rates.hip -- issue-rate probe of the integer VALU instructions the
// front end is built from (gfx950): v_add_u32, v_mul_i32_i24, v_mul_hi_i32,
// v_mad_i64_i32.  Every thread runs 8 independent dependency chains so that
// throughput, not latency, bounds the loop; 8 waves per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

template <int OP>
__global__ __launch_bounds__(256) void k(int32_t* out, int32_t seed) {
    int32_t v[8];
    int64_t w[8];
    for (int i = 0; i < 8; ++i) { v[i] = seed + threadIdx.x * 8 + i; w[i] = v[i]; }
    const int32_t c = seed | 0x12345;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(c));
            if (OP == 1) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(v[i]) : "v"(c));
            if (OP == 2) asm volatile("v_mul_hi_i32 %0, %0, %1" : "+v"(v[i]) : "v"(c));
            if (OP == 3) {
                uint64_t cc;
                asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(w[i]), "=s"(cc) : "v"(v[i]), "v"(c));
            }
        }
    }
    int64_t s = 0;
    for (int i = 0; i < 8; ++i) s += v[i] + w[i];
    if (s == 0x7fffffff) out[0] = (int32_t)s;
}

int main() {
    int cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    int32_t* out;
    hipMalloc(&out, 4);
    const int blocks = cus * 8;   // 8 waves per SIMD (4 SIMDs x 8 = 32 waves per CU = 8 blocks of 4 waves)
    const char* names[4] = {"v_add_u32", "v_mul_i32_i24", "v_mul_hi_i32", "v_mad_i64_i32"};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("{\"compute_units\": %d, \"clock_khz\": %d, \"rates\": {", cus, clk);
    for (int op = 0; op < 4; ++op) {
        auto run = [&]() {
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 7);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 7);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 7);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 7);
        };
        run();
        hipDeviceSynchronize();
        hipEventRecord(a, 0);
        for (int r = 0; r < 5; ++r) run();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double lane_ops = 5.0 * blocks * 256.0 * ITERS * 8.0;
        printf("%s\"%s\": %.4g", op ? ", " : "", names[op], lane_ops / (ms * 1e-3));
    }
    printf("}, \"unit\": \"lane-ops/s\"}\n");
    return 0;
}
