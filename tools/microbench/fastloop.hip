// Microbenchmark: cycles per iteration of the geodesic fast step for ONE
// wave alone on the GPU (the critical path of sr_integrate_kernel is a single
// long-running wave). Variants add the pieces of the step one at a time.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off fastloop.hip -o fastloop && ./fastloop
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float ddu(float u) { return -u * (1.0f - 1.5f * u); }

template <int V>
__global__ void kern(const float4* __restrict__ tbl, int n, float* out, unsigned long long* cyc) {
    float u = 0.3f + threadIdx.x * 1e-4f, du = 0.01f, rA = 1.0f / u, T = 0.0f, up = 0.0f;
    float lim = 1e30f;
    const float uf = 0.01f;
    int exits = 0;
    __syncthreads();
    const unsigned long long t0 = clock64();
    const float4* tp = tbl;
    for (int i = 0; i < n; i++) {
        const float4 e = V >= 5 ? tp[0] : tbl[0];
        const float g = V >= 5 ? tp[1].x : 1e-5f;
        float un, dun;
        if (V == 0) {  // scalar RK4
            const float h = e.x, h6 = e.y;
            const float k1 = du, l1 = ddu(u);
            const float k2 = du + 0.5f * l1 * h, l2 = ddu(u + 0.5f * k1 * h);
            const float k3 = du + 0.5f * l2 * h, l3 = ddu(u + 0.5f * k2 * h);
            const float k4 = du + l3 * h, l4 = ddu(u + k3 * h);
            un = u + h6 * (k1 + 2.0f * k2 + 2.0f * k3 + k4);
            dun = du + h6 * (l1 + 2.0f * l2 + 2.0f * l3 + l4);
        } else {
            const v2f s0 = {u, du}, hh = {e.x, e.x};
            const v2f q1 = {du, ddu(u)};
            const v2f p1 = s0 + (0.5f * q1) * hh;
            const v2f q2 = {p1.y, ddu(p1.x)};
            const v2f p2 = s0 + (0.5f * q2) * hh;
            const v2f q3 = {p2.y, ddu(p2.x)};
            const v2f p3 = s0 + q3 * hh;
            const v2f q4 = {p3.y, ddu(p3.x)};
            const v2f hs = {e.y, e.y};
            const v2f r = s0 + hs * (((q1 + 2.0f * q2) + 2.0f * q3) + q4);
            un = r.x;
            dun = r.y;
        }
        float Tn = T;
        if (V >= 2) {
            const float rB = __builtin_amdgcn_rcpf(un);
            const float dr = rB - rA;
            const float sq = __builtin_amdgcn_sqrtf(__builtin_fmaf(dr, dr, (rA * rB) * g));
            Tn = __builtin_fmaf(rA + rB, 4.0e-6f, __builtin_fmaf(sq, 1.0101f, T));
            rA = rB;
        }
        if (V >= 3) {
            if (__ballot(!(Tn < lim) || un < uf)) {
                exits++;
                lim = 2e30f;
            }
        }
        T = Tn;
        up = u;
        u = un;
        du = dun;
        tp += 2;
    }
    const unsigned long long t1 = clock64();
    out[threadIdx.x] = u + du + T + up + exits;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int V>
void run(const float4* tbl, int n, float* out, unsigned long long* cyc, const char* name) {
    unsigned long long h = 0;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(kern<V>, dim3(1), dim3(64), 0, 0, tbl, n, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, cyc, sizeof h, hipMemcpyDeviceToHost);
    }
    printf("%-40s %8.1f cycles/iteration\n", name, (double)h / n);
}

// software-pipelined: RK4 of step i+1 computed while the exit ballot of step i resolves; table prefetched 2 ahead
template <int V>
__global__ void kpipe(const float4* __restrict__ tbl, int n, float* out, unsigned long long* cyc) {
    float u = 0.3f + threadIdx.x * 1e-4f, du = 0.01f, rA = 1.0f / u, T = 0.0f, up = 0.0f;
    float lim = 1e30f;
    const float uf = 0.01f;
    int exits = 0;
    __syncthreads();
    const unsigned long long t0 = clock64();
    const float4* tp = tbl;
    auto rk4 = [&](float u, float du, float h, float h6, float& un, float& dun) {
        if (V == 1) {
            const v2f s0 = {u, du}, hh = {0.5f * h, 0.5f * h}, h1 = {h, h};
            const v2f q1 = {du, ddu(u)};
            const v2f p1 = s0 + q1 * hh;
            const v2f q2 = {p1.y, ddu(p1.x)};
            const v2f p2 = s0 + q2 * hh;
            const v2f q3 = {p2.y, ddu(p2.x)};
            const v2f p3 = s0 + q3 * h1;
            const v2f q4 = {p3.y, ddu(p3.x)};
            const v2f hs = {h6, h6};
            const v2f two = {2.0f, 2.0f};
            const v2f r = s0 + hs * (__builtin_elementwise_fma(two, q3, __builtin_elementwise_fma(two, q2, q1)) + q4);
            un = r.x;
            dun = r.y;
        } else {
            const v2f s0 = {u, du}, hh = {h, h};
            const v2f q1 = {du, ddu(u)};
            const v2f p1 = s0 + (0.5f * q1) * hh;
            const v2f q2 = {p1.y, ddu(p1.x)};
            const v2f p2 = s0 + (0.5f * q2) * hh;
            const v2f q3 = {p2.y, ddu(p2.x)};
            const v2f p3 = s0 + q3 * hh;
            const v2f q4 = {p3.y, ddu(p3.x)};
            const v2f hs = {h6, h6};
            const v2f r = s0 + hs * (((q1 + 2.0f * q2) + 2.0f * q3) + q4);
            un = r.x;
            dun = r.y;
        }
    };
    float4 e0 = tp[0], e1 = tp[2];
    float g0 = tp[1].x, g1 = tp[3].x;
    float un, dun;
    rk4(u, du, e0.x, e0.y, un, dun);
    float rB = __builtin_amdgcn_rcpf(un);
    float dr = rB - rA;
    float Tn = __builtin_fmaf(rA + rB, 4.0e-6f, __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(dr, dr, (rA * rB) * g0)), 1.0101f, T));
    for (int i = 0; i < n; i++) {
        const bool flag = !(Tn < lim) || un < uf;
        // next step (speculative)
        const float4 e2 = tp[4];
        const float g2 = tp[5].x;
        float un2, dun2;
        rk4(un, dun, e1.x, e1.y, un2, dun2);
        const float rB2 = __builtin_amdgcn_rcpf(un2);
        const float dr2 = rB2 - rB;
        const float Tn2 = __builtin_fmaf(rB + rB2, 4.0e-6f, __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(dr2, dr2, (rB * rB2) * g1)), 1.0101f, Tn));
        if (__ballot(flag)) {
            exits++;
            lim = 2e30f;
        }
        T = Tn;
        up = u;
        u = un;
        du = dun;
        rA = rB;
        un = un2;
        dun = dun2;
        rB = rB2;
        Tn = Tn2;
        e1 = e2;
        g1 = g2;
        tp += 2;
    }
    const unsigned long long t1 = clock64();
    out[threadIdx.x] = u + du + T + up + exits + rA;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int V>
void runp(const float4* tbl, int n, float* out, unsigned long long* cyc, const char* name) {
    unsigned long long h = 0;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(kpipe<V>, dim3(1), dim3(64), 0, 0, tbl, n, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, cyc, sizeof h, hipMemcpyDeviceToHost);
    }
    printf("%-40s %8.1f cycles/iteration\n", name, (double)h / n);
}

int main() {
    const int n = 4000;
    float4* tbl;
    float* out;
    unsigned long long* cyc;
    (void)hipMalloc(&tbl, sizeof(float4) * 2 * (n + 1));
    float4* h = new float4[2 * (n + 1)];
    for (int i = 0; i < 2 * (n + 1); i++) h[i] = make_float4(0.00628f, 0.00628f / 6, 0.5f, 0.5f);
    (void)hipMemcpy(tbl, h, sizeof(float4) * 2 * (n + 1), hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 64 * sizeof(float));
    (void)hipMalloc(&cyc, sizeof(unsigned long long));
    run<0>(tbl, n, out, cyc, "scalar RK4");
    run<1>(tbl, n, out, cyc, "packed RK4");
    run<2>(tbl, n, out, cyc, "packed RK4 + rcp + bound");
    run<3>(tbl, n, out, cyc, "  + ballot exit check");
    run<5>(tbl, n, out, cyc, "  + streaming table loads");
    runp<0>(tbl, n, out, cyc, "pipelined (ballot behind next RK4)");
    runp<1>(tbl, n, out, cyc, "pipelined + 0.5h / fma(2,q) RK4");
    return 0;
}
