// valu_rates2.hip -- issue cost of the VALU instruction forms the front end
// compiles to (gfx950), relative to v_add_u32: 8 independent chains per
// thread, 8 waves per SIMD, 5 timed launches; prints cycles per wave64
// instruction per SIMD at the clock measured from s_memtime over the launch.
// build: hipcc --offload-arch=gfx950 -O3 valu_rates2.hip -o valu_rates2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

#define OPS(X)                                                                                   \
    X(0, "v_add_u32", asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))                   \
    X(1, "v_sub_u32", asm volatile("v_sub_u32 %0, %1, %0" : "+v"(v[i]) : "v"(c)))                   \
    X(2, "v_ashrrev_i32", asm volatile("v_ashrrev_i32 %0, 1, %0" : "+v"(v[i])))                     \
    X(3, "v_add_lshl_u32", asm volatile("v_add_lshl_u32 %0, %0, %1, 1" : "+v"(v[i]) : "v"(c)))      \
    X(4, "v_mul_hi_i32", asm volatile("v_mul_hi_i32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))             \
    X(5, "v_mad_i64_i32", { uint64_t cc; asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(w[i]), "=s"(cc) : "v"(v[i]), "v"(c)); }) \
    X(6, "v_mul_i32_i24", asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(v[i]) : "v"(c)))           \
    X(7, "v_mul_i32_i24_sdwa", asm volatile("v_mul_i32_i24_sdwa %0, sext(%0), sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1" : "+v"(v[i]) : "v"(c))) \
    X(8, "v_permlane32_swap", asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(v[i]), "+v"(v[(i + 1) & 7]))) \
    X(9, "v_permlane16_swap", asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(v[i]), "+v"(v[(i + 1) & 7]))) \
    X(10, "v_lshl_add_u64", asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(w[i]) : "v"(w[(i + 1) & 7]))) \
    X(11, "v_ashrrev_i64", asm volatile("v_ashrrev_i64 %0, 3, %0" : "+v"(w[i])))                    \
    X(12, "v_alignbit_b32", asm volatile("v_alignbit_b32 %0, %0, %1, 15" : "+v"(v[i]) : "v"(c)))    \
    X(13, "v_med3_i32", asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(d)))    \
    X(14, "v_cndmask_b32", asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "s"(m))) \
    X(15, "v_cmp_gt_i64", { uint64_t cc; asm volatile("v_cmp_gt_i64 %0, %1, %2" : "=s"(cc) : "v"(w[i]), "v"(w[(i + 3) & 7])); acc ^= cc; }) \
    X(16, "v_mov_b64", asm volatile("v_mov_b64 %0, %1" : "=v"(w[i]) : "v"(w[(i + 1) & 7])))         \
    X(17, "v_bfe_i32", asm volatile("v_bfe_i32 %0, %0, 3, 20" : "+v"(v[i])))                       \
    X(18, "v_add3_u32", asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(d)))    \
    X(19, "v_mad_u64_u32", { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[i]), "=s"(cc) : "v"(v[i]), "v"(c)); }) \
    X(20, "v_mul_lo_u32", asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))            \
    X(21, "v_pk_add_f32", asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(w[i]) : "v"(w[(i + 1) & 7])))

#define NOPS 22

template <int OP>
__global__ __launch_bounds__(256) void k(int32_t* out, int32_t seed, long long* clk) {
    int32_t v[8];
    int64_t w[8];
    for (int i = 0; i < 8; ++i) { v[i] = seed + threadIdx.x * 8 + i; w[i] = v[i]; }
    const int32_t c = seed | 0x12345, d = seed ^ 0x7777;
    const uint64_t m = 0x5555555555555555ull;
    uint64_t acc = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#define CASE(n, name, body) if (OP == n) body;
            OPS(CASE)
#undef CASE
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    int64_t s = (int64_t)acc;
    for (int i = 0; i < 8; ++i) s += v[i] + w[i];
    if (s == 0x7fffffff) out[0] = (int32_t)s;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[OP] = t1 - t0;
}

template <int OP>
static void launch(int blocks, int32_t* out, long long* clk) {
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 7, clk);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int32_t* out;
    long long* clk;
    hipMalloc(&out, 4);
    hipMalloc(&clk, 64 * 8);
    const int blocks = cus * 8;   // 8 waves per SIMD
    const char* names[NOPS];
#define NAME(n, name, body) names[n] = name;
    OPS(NAME)
#undef NAME
    typedef void (*L)(int, int32_t*, long long*);
    L fns[NOPS] = {launch<0>, launch<1>, launch<2>, launch<3>, launch<4>, launch<5>, launch<6>, launch<7>,
                   launch<8>, launch<9>, launch<10>, launch<11>, launch<12>, launch<13>, launch<14>, launch<15>,
                   launch<16>, launch<17>, launch<18>, launch<19>, launch<20>, launch<21>};
    printf("{\"compute_units\": %d, \"note\": \"SIMD cycles per wave64 instruction (8 waves/SIMD, 8 chains each); cycles from s_memtime of one wave\", \"cycles\": {", cus);
    for (int op = 0; op < NOPS; ++op) {
        fns[op](blocks, out, clk);
        hipDeviceSynchronize();
        fns[op](blocks, out, clk);
        hipDeviceSynchronize();
        long long c = 0;
        hipMemcpy(&c, clk + op, 8, hipMemcpyDeviceToHost);
        // one wave's span covers 8 waves/SIMD x ITERS x 8 instructions on its SIMD
        const double per = (double)c / (8.0 * ITERS * 8.0);
        printf("%s\"%s\": %.2f", op ? ", " : "", names[op], per);
    }
    printf("}}\n");
    return 0;
}
