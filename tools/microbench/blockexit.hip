// Microbenchmark: the fast step's exit test per step (production: a ballot
// and a branch after every step, kernels/geodesic.hip integrate) against one
// exit test per three-step block (the three steps' conditions ORed, one
// branch): without the branches between them, step k's chord bound (rcp,
// sqrt) and ballot can issue under step k + 1's RK4 chain. Throughput over
// the whole GPU and the per-wave latency at 1 wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off blockexit.hip -o blockexit && ./blockexit
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float sr_v4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) sr_v4f cf4;

__device__ __forceinline__ float ddu(float u) { return -u * (1.0f - 1.5f * u); }

__device__ __forceinline__ void rk4_1(float u, float du, float h, float hh, float h6, float& un, float& dun) {
    const v2f s0 = {u, du};
    const v2f H1 = {h, h}, H2 = {hh, hh}, two = {2.0f, 2.0f};
    const v2f q1 = {du, ddu(u)};
    v2f p1 = s0 + q1 * H2;
    p1.x = ddu(p1.x);
    v2f p2 = s0 + p1.yx * H2;
    p2.x = ddu(p2.x);
    v2f p3 = s0 + p2.yx * H1;
    p3.x = ddu(p3.x);
    const v2f hs = {h6, h6};
    const v2f r = s0 + hs * (__builtin_elementwise_fma(two, p2.yx, __builtin_elementwise_fma(two, p1.yx, q1)) + p3.yx);
    un = r.x;
    dun = r.y;
}

// MODE 0: ballot + branch per step; MODE 1: one ballot (OR of the three
// steps' conditions) per block; MODE 2: three ballots ORed in SGPRs, one branch
template <int MODE>
__global__ __launch_bounds__(64) void kern(const float4* __restrict__ tbl, int n, float* out, int* hits) {
    extern __shared__ float pad[];
    const int t = blockIdx.x * 64 + threadIdx.x;
    const float lim = 1e30f, uf = 0.01f;
    const cf4* tp = (const cf4*)tbl;
    sr_v4f e = tp[0], e1 = tp[1];
    float u = 0.3f + (t & 1023) * 1e-5f, du = 0.01f, rA = 1.0f / u, T = 0.0f;
    int exits = 0;
    for (int i = 0; i < n; i += 3) {
        sr_v4f nx[6];
#pragma unroll
        for (int k = 0; k < 6; k++) nx[k] = tp[2 + k];
        __builtin_amdgcn_sched_barrier(0);
        bool any = false;
        unsigned long long m = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            float a, b;
            rk4_1(u, du, e.x, e1.y, e.y, a, b);
            const float r = __builtin_amdgcn_rcpf(a);
            const float dr = r - rA;
            const float sq = __builtin_amdgcn_sqrtf(__builtin_fmaf(dr, dr, (rA * r) * e1.x));
            const float Tn = __builtin_fmaf(sq, e1.z, T);
            const bool c = !(Tn < lim) || a < uf;
            if (MODE == 0) {
                if (__ballot(c)) {
                    exits++;
                    if (exits > n) break;
                }
            } else if (MODE == 1) {
                any = any || c;
            } else {
                m |= __ballot(c);
            }
            T = Tn;
            u = a;
            du = b;
            rA = r;
            e = nx[2 * k];
            e1 = nx[2 * k + 1];
        }
        if (MODE == 1 && __ballot(any)) {
            exits++;
            if (exits > n) break;
        }
        if (MODE == 2 && m) {
            exits++;
            if (exits > n) break;
        }
        tp += 6;
    }
    out[t] = u + du + T;
    if (exits && threadIdx.x == 0) atomicAdd(hits, exits);
    if (threadIdx.x == 0 && n < 0) pad[0] = 1.0f;
}

template <int MODE>
double run(const float4* tbl, int n, float* out, int* hits, int waves_per_simd, int cus, int rounds, double* ms_out) {
    const int blocks = cus * 4 * waves_per_simd * rounds;
    const size_t lds = (160 * 1024) / (4 * waves_per_simd) - 256;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(64), lds, 0, tbl, n, out, hits);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;
    }
    *ms_out = best;
    return (double)blocks * 64 * n / (best * 1e-3) / 1e12;  // T ray-steps / s
}

int main() {
    const int n = 2001;
    float4* tbl;
    float* out;
    int* hits;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    (void)hipMalloc(&tbl, sizeof(float4) * 2 * (n + 8));
    float4* h = new float4[2 * (n + 8)];
    for (int i = 0; i < n + 8; i++) {
        const float s = 12.566371f / n;
        h[2 * i] = make_float4(s, s / 6, 0.5f, 0.5f);
        h[2 * i + 1] = make_float4(1e-5f, 0.5f * s, 1.0102f, 0.0f);
    }
    (void)hipMemcpy(tbl, h, sizeof(float4) * 2 * (n + 8), hipMemcpyHostToDevice);
    (void)hipMalloc(&out, (size_t)cus * 4 * 8 * 4 * 64 * sizeof(float));
    (void)hipMalloc(&hits, sizeof(int));
    (void)hipMemset(hits, 0, sizeof(int));
    printf("{\"cus\": %d, \"steps\": %d, \"results\": [", cus, n);
    bool first = true;
    for (int w : {1, 2, 4, 6, 8}) {
        double ms0, ms1, ms2;
        const int rounds = w == 1 ? 1 : 4;
        const double t0 = run<0>(tbl, n, out, hits, w, cus, rounds, &ms0);
        const double t1 = run<1>(tbl, n, out, hits, w, cus, rounds, &ms1);
        const double t2 = run<2>(tbl, n, out, hits, w, cus, rounds, &ms2);
        // at one wave per SIMD the kernel time is one wave's latency: cycles per step at 2.4 GHz
        printf("%s{\"waves_per_simd\": %d, \"per_step_Tsteps\": %.4f, \"per_block_or_Tsteps\": %.4f, "
               "\"per_block_3ballots_Tsteps\": %.4f, \"ms\": [%.4f, %.4f, %.4f]}",
               first ? "" : ", ", w, t0, t1, t2, ms0, ms1, ms2);
        first = false;
    }
    int hh = 0;
    (void)hipMemcpy(&hh, hits, sizeof(int), hipMemcpyDeviceToHost);
    printf("], \"exits\": %d}\n", hh);
    return 0;
}
