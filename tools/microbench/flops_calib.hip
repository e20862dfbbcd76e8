// flops_calib.hip — calibrates rocprofv3's SQ_INSTS_VALU_FLOPS_FP32 (and the
// per-type SQ_INSTS_VALU_*_F32 counters) on gfx950 against kernels whose
// FP32 work is known exactly: fixed counts of v_fma_f32 / v_pk_fma_f32 /
// v_add_f32 / v_mul_f32 / v_rcp_f32 per lane, all lanes or half of them
// active. bench.py turns the counters of the geodesic kernel into executed
// FLOP with the factors this measures (tools/pmc_flops.py).
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/flops_calib.hip -o tools/microbench/flops_calib
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 ... -- tools/microbench/flops_calib
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITERS 256
typedef float v2f __attribute__((ext_vector_type(2)));

// mode: 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_add_f32, 3 v_mul_f32, 4 v_rcp_f32
template <int MODE, bool HALF>
__global__ __launch_bounds__(256) void calib(float* out, float b, float c) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1.0f, a2 = a0 + 2.0f, a3 = a0 + 3.0f;
    v2f p0 = {a0, a1}, p1 = {a2, a3};
    const v2f pb = {b, b}, pc = {c, c};
    if (!HALF || (threadIdx.x & 1)) {
        for (int i = 0; i < ITERS; i++) {
            if (MODE == 0) {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));
            } else if (MODE == 1) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p0) : "v"(pb), "v"(pc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p1) : "v"(pb), "v"(pc));
            } else if (MODE == 2) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a1) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a2) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a3) : "v"(b));
            } else if (MODE == 3) {
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a0) : "v"(b));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a1) : "v"(b));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a2) : "v"(b));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a3) : "v"(b));
            } else {
                asm volatile("v_rcp_f32 %0, %0" : "+v"(a0));
                asm volatile("v_rcp_f32 %0, %0" : "+v"(a1));
                asm volatile("v_rcp_f32 %0, %0" : "+v"(a2));
                asm volatile("v_rcp_f32 %0, %0" : "+v"(a3));
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + p0.x + p0.y + p1.x + p1.y;
}

int main() {
    const int blocks = 1024;
    float* d = nullptr;
    if (hipMalloc(&d, blocks * 256 * sizeof(float)) != hipSuccess) return 1;
    // the known work per launch, per lane-instruction accounting
    const double lanes = blocks * 256.0;
    printf("lanes %.0f iters %d; per active lane: 4*ITERS instr (pk: 2*ITERS)\n", lanes, ITERS);
#define RUN(M, H, name)                                                          \
    hipLaunchKernelGGL((calib<M, H>), dim3(blocks), dim3(256), 0, 0, d, 1.0001f, 0.5f); \
    if (hipDeviceSynchronize() != hipSuccess) return 2;                           \
    printf("%s\n", name);
    RUN(0, false, "fma_f32 full: 2048 flop/lane");
    RUN(0, true, "fma_f32 half: 2048 flop/active lane, half the lanes");
    RUN(1, false, "pk_fma_f32 full: 2048 flop/lane");
    RUN(2, false, "add_f32 full: 1024 flop/lane");
    RUN(3, false, "mul_f32 full: 1024 flop/lane");
    RUN(4, false, "rcp_f32 full: 1024 trans/lane");
    (void)hipFree(d);
    return 0;
}
