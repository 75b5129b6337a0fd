// ubench_valu.hip -- measured issue rate of the int32 VALU instructions the
// SHA-256 kernel is made of, on the whole chip, plus the shader clock under
// that load (s_memtime / s_memrealtime).  Build: see tools/Makefile.ubench.
//
// Each lane runs 8 independent dependency chains of one instruction
// (inline asm so nothing folds), 8 waves per SIMD, every CU busy.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHAINS 8
#define ITERS 8192
#define UNROLL 4

#define OP8_(OPSTR)                                                                                            \
    asm volatile(OPSTR : "+v"(a0) : "v"(b)); asm volatile(OPSTR : "+v"(a1) : "v"(b));                         \
    asm volatile(OPSTR : "+v"(a2) : "v"(b)); asm volatile(OPSTR : "+v"(a3) : "v"(b));                         \
    asm volatile(OPSTR : "+v"(a4) : "v"(b)); asm volatile(OPSTR : "+v"(a5) : "v"(b));                         \
    asm volatile(OPSTR : "+v"(a6) : "v"(b)); asm volatile(OPSTR : "+v"(a7) : "v"(b));
#define OP8(OPSTR) OP8_(OPSTR) OP8_(OPSTR) OP8_(OPSTR) OP8_(OPSTR)

template <int OP>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned long long* clk, unsigned seed) {
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (OP == 0) { OP8("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 1) { OP8("v_add_u32_e64 %0, %0, %1") }
        if constexpr (OP == 2) { OP8("v_add3_u32 %0, %0, %1, %0") }
        if constexpr (OP == 3) { OP8("v_alignbit_b32 %0, %0, %1, 7") }
        if constexpr (OP == 4) { OP8("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96") }
        if constexpr (OP == 5) { OP8("v_xor_b32 %0, %0, %1") }
        if constexpr (OP == 6) { OP8("v_or_b32 %0, %0, %1") }
        if constexpr (OP == 7) { OP8("v_and_b32 %0, %0, %1") }
        if constexpr (OP == 8) { OP8("v_lshrrev_b32 %0, 3, %0") }
        if constexpr (OP == 9) { OP8("v_lshlrev_b32 %0, 3, %0") }
        if constexpr (OP == 10) { OP8("v_lshrrev_b32_e64 %0, %1, %0") }
        if constexpr (OP == 11) { OP8("v_sub_u32 %0, %0, %1") }
        if constexpr (OP == 12) { OP8("v_cndmask_b32 %0, %0, %1, vcc") }
        if constexpr (OP == 13) { OP8("v_mov_b32 %0, %1") }
        if constexpr (OP == 14) { OP8("v_not_b32 %0, %0") }
        if constexpr (OP == 15) { OP8("v_bfe_u32 %0, %0, %1, 5") }
        if constexpr (OP == 16) { OP8("v_lshrrev_b64 v[40:41], 3, v[40:41]") }
        if constexpr (OP == 17) { OP8("v_mul_u32_u24 %0, %0, %1") }
        if constexpr (OP == 18) { OP8("v_mul_lo_u32 %0, %0, %1") }
        if constexpr (OP == 19) { OP8("v_max_u32 %0, %0, %1") }
        if constexpr (OP == 20) { OP8("v_pk_fma_f32 v[40:41], v[40:41], v[42:43], v[40:41]") }
        if constexpr (OP == 21) { OP8("v_pk_add_f32 v[40:41], v[40:41], v[42:43]") }
        if constexpr (OP == 22) { OP8("v_pk_mov_b32 v[40:41], v[42:43], v[40:41] op_sel:[0,1]") }
        if constexpr (OP == 23) { OP8("v_add_f32 %0, %0, %1") }
        if constexpr (OP == 24) { OP8("v_fma_f32 %0, %0, %1, %0") }
        if constexpr (OP == 25) { OP8("v_bitop3_b16 %0, %0, %1, %0 bitop3:0x96") }
        if constexpr (OP == 26) { OP8("v_add_u16 %0, %0, %1") }
        if constexpr (OP == 27) { OP8("v_alignbit_b32 %0, %0, %0, 7") }
        if constexpr (OP == 28) { OP8("v_add_u32 %0, s8, %0") }
        if constexpr (OP == 29) { OP8("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD") }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static const char* names[] = {"v_add_u32", "v_add_u32_e64", "v_add3_u32", "v_alignbit_b32", "v_bitop3_b32", "v_xor_b32", "v_or_b32", "v_and_b32", "v_lshrrev_b32", "v_lshlrev_b32", "v_lshrrev_b32_e64v", "v_sub_u32", "v_cndmask_b32", "v_mov_b32", "v_not_b32", "v_bfe_u32", "v_lshrrev_b64", "v_mul_u32_u24", "v_mul_lo_u32", "v_max_u32", "v_pk_fma_f32", "v_pk_add_f32", "v_pk_mov_b32", "v_add_f32", "v_fma_f32", "v_bitop3_b16", "v_add_u16", "v_alignbit_s", "v_add_u32_sgpr", "v_xor_sdwa"};
static const int per_op[] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1};

template <int OP>
void run(int grid, int block) {
    unsigned* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)grid * block * 4);
    hipMalloc(&clk, (size_t)grid * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<OP><<<grid, block>>>(out, clk, 1);  // warm
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        kern<OP><<<grid, block>>>(out, clk, r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    unsigned long long* h = (unsigned long long*)malloc((size_t)grid * 16);
    hipMemcpy(h, clk, (size_t)grid * 16, hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    for (int i = 0; i < grid; ++i) {
        cyc += h[2 * i];
        real += h[2 * i + 1];
    }
    double ghz = (cyc / grid) / ((real / grid) / 100e6) / 1e9;  // memrealtime = 100 MHz
    double lane_ops = (double)grid * block * ITERS * UNROLL * CHAINS * per_op[OP];
    double tops = lane_ops / (best * 1e-3) / 1e12;
    // cycles per wave-instruction per SIMD: (wall cycles * 4 SIMD * CUs) / wave-instrs
    printf("%-16s %8.3f ms  %7.2f T lane-ops/s  in-kernel clock %.3f GHz  -> %.2f lane-ops/clk/CU\n", names[OP],
           best, tops, ghz, tops * 1e12 / (ghz * 1e9) / 256.0);
    free(h);
    hipFree(out);
    hipFree(clk);
}

int main(int argc, char** argv) {
    int bpc = argc > 1 ? atoi(argv[1]) : 8;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int grid = p.multiProcessorCount * bpc;
    printf("%s, %d CUs, grid %d x 256\n", p.gcnArchName, p.multiProcessorCount, grid);
    run<0>(grid, 256);
    run<1>(grid, 256);
    run<2>(grid, 256);
    run<3>(grid, 256);
    run<4>(grid, 256);
    run<5>(grid, 256);
    run<6>(grid, 256);
    run<7>(grid, 256);
    run<8>(grid, 256);
    run<9>(grid, 256);
    run<10>(grid, 256);
    run<11>(grid, 256);
    run<12>(grid, 256);
    run<13>(grid, 256);
    run<14>(grid, 256);
    run<15>(grid, 256);
    run<16>(grid, 256);
    run<17>(grid, 256);
    run<18>(grid, 256);
    run<19>(grid, 256);
    run<20>(grid, 256);
    run<21>(grid, 256);
    run<22>(grid, 256);
    run<23>(grid, 256);
    run<24>(grid, 256);
    run<25>(grid, 256);
    run<26>(grid, 256);
    run<27>(grid, 256);
    run<28>(grid, 256);
    run<29>(grid, 256);
    return 0;
}
