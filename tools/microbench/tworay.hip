// Microbenchmark: THROUGHPUT of the geodesic fast step over the whole GPU,
// one ray per lane (the production form: (u, u') packed pairs) against two
// rays per lane whose RK4 runs as packed pairs ACROSS the rays ((uA, uB),
// (u'A, u'B)): the same IEEE operations per ray, about 1.5x fewer VALU
// instructions per ray-step and two independent dependency chains per lane.
// Occupancy is pinned with dynamic LDS (waves per SIMD = argv).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tworay.hip -o tworay && ./tworay
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float sr_v4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) sr_v4f cf4;

__device__ __forceinline__ float ddu(float u) { return -u * (1.0f - 1.5f * u); }
__device__ __forceinline__ v2f ddu2(v2f u) {
    const v2f k = {1.5f, 1.5f}, one = {1.0f, 1.0f};
    return -u * (one - k * u);
}

// one ray per lane: production RK4 (kernels/geodesic.hip rk4_step)
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

// two rays per lane: u = (uA, uB), du = (u'A, u'B)
__device__ __forceinline__ void rk4_2(v2f u, v2f du, float h, float hh, float h6, v2f& un, v2f& dun) {
    const v2f H1 = {h, h}, H2 = {hh, hh}, two = {2.0f, 2.0f}, HS = {h6, h6};
    const v2f k1 = du, l1 = ddu2(u);
    const v2f k2 = du + l1 * H2, l2 = ddu2(u + k1 * H2);
    const v2f k3 = du + l2 * H2, l3 = ddu2(u + k2 * H2);
    const v2f k4 = du + l3 * H1, l4 = ddu2(u + k3 * H1);
    un = u + HS * (__builtin_elementwise_fma(two, k3, __builtin_elementwise_fma(two, k2, k1)) + k4);
    dun = du + HS * (__builtin_elementwise_fma(two, l3, __builtin_elementwise_fma(two, l2, l1)) + l4);
}

template <int RAYS>
__global__ __launch_bounds__(64) void kern(const float4* __restrict__ tbl, int n, float* out) {
    extern __shared__ float pad[];
    const int t = blockIdx.x * 64 + threadIdx.x;
    const float lim = 1e30f, uf = 0.01f;
    int exits = 0;
    const cf4* tp = (const cf4*)tbl;
    if (RAYS == 1) {
        float u = 0.3f + (t & 1023) * 1e-5f, du = 0.01f, rA = 1.0f / u, T = 0.0f;
        for (int i = 0; i < n; i++) {
            const sr_v4f e = tp[0], e1 = tp[1];
            float un, dun;
            rk4_1(u, du, e.x, e1.y, e.y, un, dun);
            const float rB = __builtin_amdgcn_rcpf(un);
            const float dr = rB - rA;
            const float sq = __builtin_amdgcn_sqrtf(__builtin_fmaf(dr, dr, (rA * rB) * e1.x));
            const float Tn = __builtin_fmaf(sq, e1.z, T);
            if (__ballot(!(Tn < lim) || un < uf)) exits++;
            T = Tn;
            u = un;
            du = dun;
            rA = rB;
            tp += 2;
        }
        out[t] = u + du + T + exits;
    } else {
        v2f u = {0.3f + (t & 1023) * 1e-5f, 0.31f + (t & 1023) * 1e-5f}, du = {0.01f, 0.012f};
        v2f rA = {1.0f / u.x, 1.0f / u.y}, T = {0.0f, 0.0f};
        for (int i = 0; i < n; i++) {
            const sr_v4f e = tp[0], e1 = tp[1];
            v2f un, dun;
            rk4_2(u, du, e.x, e1.y, e.y, un, dun);
            const v2f rB = {__builtin_amdgcn_rcpf(un.x), __builtin_amdgcn_rcpf(un.y)};
            const v2f dr = rB - rA;
            const v2f G = {e1.x, e1.x}, K = {e1.z, e1.z};
            const v2f x = __builtin_elementwise_fma(dr, dr, (rA * rB) * G);
            const v2f sq = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
            const v2f Tn = __builtin_elementwise_fma(sq, K, T);
            if (__ballot(!(Tn.x < lim) || un.x < uf || !(Tn.y < lim) || un.y < uf)) exits++;
            T = Tn;
            u = un;
            du = dun;
            rA = rB;
            tp += 2;
        }
        out[t] = u.x + u.y + du.x + du.y + T.x + T.y + exits;
    }
    if (threadIdx.x == 0 && n < 0) pad[0] = 1.0f;
}

// The production fast loop's shape (kernels/geodesic.hip integrate): three
// steps per iteration, the next three steps' table entries loaded together at
// the iteration's top, an exit ballot per step.
template <int RAYS>
__global__ __launch_bounds__(64) void kern3(const float4* __restrict__ tbl, int n, float* out) {
    extern __shared__ float pad[];
    const int t = blockIdx.x * 64 + threadIdx.x;
    const float lim = 1e30f, uf = 0.01f;
    int exits = 0;
    const cf4* tp = (const cf4*)tbl;
    sr_v4f e = tp[0], e1 = tp[1];
    v2f u, du, rA, T;
    if (RAYS == 1) {
        u = {0.3f + (t & 1023) * 1e-5f, 0.0f};
        du = {0.01f, 0.0f};
    } else {
        u = {0.3f + (t & 1023) * 1e-5f, 0.31f + (t & 1023) * 1e-5f};
        du = {0.01f, 0.012f};
    }
    rA = {1.0f / u.x, 1.0f / u.y};
    T = {0.0f, 0.0f};
    for (int i = 0; i < n; i += 3) {
        sr_v4f nx[6];
#pragma unroll
        for (int k = 0; k < 6; k++) nx[k] = tp[2 + k];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            v2f un, dun, rB, Tn;
            if (RAYS == 1) {
                float a, b;
                rk4_1(u.x, du.x, e.x, e1.y, e.y, a, b);
                un = {a, 0.0f};
                dun = {b, 0.0f};
                const float r = __builtin_amdgcn_rcpf(a);
                const float dr = r - rA.x;
                const float sq = __builtin_amdgcn_sqrtf(__builtin_fmaf(dr, dr, (rA.x * r) * e1.x));
                rB = {r, 0.0f};
                Tn = {__builtin_fmaf(sq, e1.z, T.x), 0.0f};
                if (__ballot(!(Tn.x < lim) || a < uf)) exits++;
            } else {
                rk4_2(u, du, e.x, e1.y, e.y, un, dun);
                rB = {__builtin_amdgcn_rcpf(un.x), __builtin_amdgcn_rcpf(un.y)};
                const v2f dr = rB - rA;
                const v2f G = {e1.x, e1.x}, K = {e1.z, e1.z};
                const v2f x = __builtin_elementwise_fma(dr, dr, (rA * rB) * G);
                const v2f sq = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
                Tn = __builtin_elementwise_fma(sq, K, T);
                if (__ballot(!(Tn.x < lim) || un.x < uf || !(Tn.y < lim) || un.y < uf)) exits++;
            }
            T = Tn;
            u = un;
            du = dun;
            rA = rB;
            e = nx[2 * k];
            e1 = nx[2 * k + 1];
        }
        tp += 6;
    }
    out[t] = u.x + u.y + du.x + du.y + T.x + T.y + exits;
    if (threadIdx.x == 0 && n < 0) pad[0] = 1.0f;
}

template <int RAYS, bool THREE>
double run(const float4* tbl, int n, float* out, int waves_per_simd, int cus) {
    const int blocks = cus * 4 * waves_per_simd * 4;  // 4 rounds of full occupancy
    const size_t lds = (160 * 1024) / (4 * waves_per_simd) - 256;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
        (void)hipEventRecord(a, 0);
        if (THREE) hipLaunchKernelGGL(kern3<RAYS>, dim3(blocks), dim3(64), lds, 0, tbl, n, out);
        else hipLaunchKernelGGL(kern<RAYS>, dim3(blocks), dim3(64), lds, 0, tbl, n, out);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;
    }
    const double ray_steps = (double)blocks * 64 * RAYS * n;
    return ray_steps / (best * 1e-3) / 1e12;  // T ray-steps / s
}

int main(int argc, char** argv) {
    const int n = 2000;
    float4* tbl;
    float* out;
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
    printf("{\"cus\": %d, \"steps\": %d, \"results\": [", cus, n);
    bool first = true;
    for (int w : {2, 3, 4, 5, 6, 8}) {
        const double one = run<1, false>(tbl, n, out, w, cus), two = run<2, false>(tbl, n, out, w, cus);
        const double one3 = run<1, true>(tbl, n, out, w, cus), two3 = run<2, true>(tbl, n, out, w, cus);
        printf("%s{\"waves_per_simd\": %d, \"one_ray_Tsteps\": %.4f, \"two_rays_Tsteps\": %.4f, "
               "\"one_ray_3step_prefetch_Tsteps\": %.4f, \"two_rays_3step_prefetch_Tsteps\": %.4f}",
               first ? "" : ", ", w, one, two, one3, two3);
        first = false;
    }
    printf("]}\n");
    return 0;
}
