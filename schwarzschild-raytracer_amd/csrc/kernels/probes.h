// probes.h - the measurement hooks of the integrate kernel (SR_STATS*,
// SR_PROF, SR_LANE_MASK, SR_STATS_FIRE builds: tools/stats_frame.py,
// stats_bh.py, stats_dir.py, prof_waves.py, lane_mask.py, built by
// tools/build_variant.sh). Round 6 gathered them here from the
// kernel's control flow: geodesic.hip calls them at a few sites, and in the
// shipping build every hook is an empty inline function, an empty struct or a
// ((void)0) macro, so the kernel's machine code is the same as without them
// (make isa, diffed when this file was split off). Included once, by
// geodesic.hip, before the kernel code.
#ifndef SR_PROBES_H
#define SR_PROBES_H

// budget slots 0 .. 8 have their own counters in measurement builds
#define SR_STATS_SLOTS 9
#ifdef SR_STATS
// Measurement builds only: wave-level event counters (tools/stats_frame.py).
//   0 wave-steps  1 budget events  2..10 slot j reached (exact chord)
//   11 -  12 exact object tests run  13 lane-steps  14..22 slot j spent
__device__ unsigned long long sr_stats[64];
// per-wave [start, end] s_memrealtime (100 MHz) of sr_integrate_kernel, by wave index
#define SR_WAVE_LOG (1 << 17)
#define SR_WAVE_REC 16  // t0, t1, max steps, events << 32 | exact chords, reach count of slots 0..8
__device__ unsigned long long sr_wave_t[SR_WAVE_REC * SR_WAVE_LOG];
__device__ __forceinline__ void stat_add(int k, unsigned long long v) {
    const unsigned long long act = __ballot(1);
    if ((int)__lane_id() == __builtin_ctzll(act)) atomicAdd(&sr_stats[k], v);
}
#ifdef SR_STATS_NOCOUNT  // timeline only: the counters' atomics distort it
#define SR_STAT(k, v) ((void)0)
#else
#define SR_STAT(k, v) stat_add(k, v)
#endif
#else
#define SR_STAT(k, v) ((void)0)
#endif

#ifdef SR_LANE_MASK
// Latency experiments only: a per-pixel keep mask (device pointer) over the full frame
__device__ const uint8_t* sr_lane_mask;
#endif

#ifdef SR_PROF
// Measurement builds only (tools/prof_waves.py): per-wave shader-clock cycles
// by section of the step loop, wave-uniform accumulators (no per-lane state,
// so the build keeps the production register allocation as far as possible).
//   0 fast loop  1 reseeds  2 slow-path entry + approximate chord  3 budget events phase 1
//   4 exact chord + intersect  5 hit classification + log  6 budget events phase 2  7 wave total
#define SR_PROF_N 24  // 0-6 sections, 7 wave total | max steps << 48, 8-15 re-anchors of budget slots 0-7,
                      // 22 budget_init, 23 kernel start to integrate (launch code, pixel, ray set-up),
                      // 16 budget events, 17 events spending only slot 0, 18 lanes spending slot 0 (sum),
                      // 19 slow-path entries, 20 event phase 1 up to the spent ballots (the rest
                      // in 3), 21 slow-path tail + top of the step loop (2: exit to the event)
__device__ unsigned long long sr_prof[SR_PROF_N * (1 << 17)];
#define SR_PT(k)                                                      \
    do {                                                              \
        const unsigned t_ = (unsigned)clock64();                      \
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) r.prof[k] += t_ - prof_t_; \
        prof_t_ = t_;                                                 \
    } while (0)
// the same inside budget_event (accumulators reached through the Budget)
#define SR_PTB(k)                                                     \
    do {                                                              \
        const unsigned t_ = (unsigned)clock64();                      \
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) bs.prof[k] += t_ - *bs.pt; \
        *bs.pt = t_;                                                  \
    } while (0)
#else
#define SR_PT(k) ((void)0)
#define SR_PTB(k) ((void)0)
#endif

// SR_PROBE(statements): a hook site in geodesic.hip. It expands to nothing
// unless a measurement build is selected, so the shipping kernel's source is
// token for token what it was without the hooks (the probes' argument
// expressions are not even evaluated).
#if defined(SR_STATS) || defined(SR_PROF) || defined(SR_LANE_MASK) || defined(SR_STATS_FIRE)
#define SR_PROBE(...) __VA_ARGS__
#else
#define SR_PROBE(...)
#endif
// SR_TRACE (with SR_LANE_MASK, one unmasked pixel): device printf of the
// slow path's steps, events and hits of the rays that run (post-mortems)
#ifdef SR_TRACE
// (inside integrate: I = the integrate kernel's pass, R = sr_resume_kernel's; the thread)
#define SR_TRACE_AT(fmt, ...) printf("%c%d " fmt, RECORD ? 'I' : 'R', (int)threadIdx.x, __VA_ARGS__)
#else
#define SR_TRACE_AT(...)
#endif
// the first active lane of the wave (the one that updates wave-level accumulators)
#define SR_LEAD() ((int)(threadIdx.x & 63) == (int)__builtin_ctzll(__ballot(1)))
// a counter only the default statistics build keeps (the SR_STATS_BH / _DIR
// builds reuse its indices), and the step-histogram build's own ones
#if defined(SR_STATS) && !defined(SR_STATS_BH) && !defined(SR_STATS_DIR)
#define SR_STAT_MAIN(k, v) SR_STAT(k, v)
#else
#define SR_STAT_MAIN(k, v) ((void)0)
#endif
#ifdef SR_STATS_STEPHIST
#define SR_STAT_STEPHIST(k, v) SR_STAT(k, v)
#else
#define SR_STAT_STEPHIST(k, v) ((void)0)
#endif

#ifdef SR_PROF
// a wave-level accumulator of the section cycles' build (acc: r.prof / bs.prof)
#define SR_PROF_BUMP(acc, k, v) \
    do {                        \
        if (SR_LEAD()) (acc)[k] += (v); \
    } while (0)
// integrate(): the clock before budget_init, then the step loop's section clock (SR_PT)
#define SR_PROF_CLOCK(name) const unsigned name = (unsigned)clock64()
#define SR_PROF_LOOP_START(r, bs, t_init)            \
    unsigned prof_t_ = (unsigned)clock64();          \
    (bs).prof = (r).prof;                            \
    (bs).pt = &prof_t_;                              \
    if (SR_LEAD()) (r).prof[22] += prof_t_ - (t_init)
#define SR_PROBE_BUDGET_PROF \
    unsigned* prof;          \
    unsigned* pt;
#define SR_PROBE_RAY_PROF unsigned* prof;  // the wave's section accumulators in LDS
#else
#define SR_PROF_BUMP(acc, k, v) ((void)0)
#define SR_PROF_CLOCK(name) ((void)0)
#define SR_PROF_LOOP_START(r, bs, t_init) ((void)0)
#define SR_PROBE_BUDGET_PROF
#define SR_PROBE_RAY_PROF
#endif
#ifdef SR_STATS_FIRE  // steps that ran any exact test (the count replaces r.steps)
#define SR_PROBE_BUDGET_FIRE int fires;
#else
#define SR_PROBE_BUDGET_FIRE
#endif
#ifdef SR_STATS
#define SR_PROBE_RAY_STATS \
    int ev, mat;  /* budget events, exact chords */ \
    int rc[SR_STATS_SLOTS];
#else
#define SR_PROBE_RAY_STATS
#endif
// the Budget's and the Ray's measurement fields
#define SR_PROBE_BUDGET_FIELDS SR_PROBE_BUDGET_FIRE SR_PROBE_BUDGET_PROF
#define SR_PROBE_RAY_FIELDS SR_PROBE_RAY_PROF SR_PROBE_RAY_STATS

// ---- per ray -------------------------------------------------------------
template <class R>
__device__ __forceinline__ void probe_ray_init(R& r) {
#ifdef SR_STATS
    r.ev = 0;
    r.mat = 0;
    for (int j = 0; j < SR_STATS_SLOTS; j++) r.rc[j] = 0;
#else
    (void)r;
#endif
}
// an exact chord of the step loop
template <class R>
__device__ __forceinline__ void probe_exact_chord(R& r) {
#ifdef SR_STATS
    r.mat++;
#else
    (void)r;
#endif
}
// the slots an event found reachable (exact chords follow)
template <class R>
__device__ __forceinline__ void probe_reach(R& r, uint32_t reach) {
#ifdef SR_STATS
    for (uint32_t c = reach & 0x1ffu; c; c &= c - 1) SR_STAT(2 + __builtin_ctz(c), 1);
#pragma unroll
    for (int j = 0; j < SR_STATS_SLOTS; j++) r.rc[j] += (reach >> j) & 1u;
#else
    (void)r;
    (void)reach;
#endif
}

// ---- the step loop's own state (integrate) -------------------------------
struct LoopProbe {
#ifdef SR_STATS
    int last_ev, near_run;  // the wave's previous event step, run of back-to-back events
    __device__ explicit LoopProbe(int i) : last_ev(i), near_run(0) {}
#else
    __device__ explicit LoopProbe(int) {}
#endif
};
// SR_STATS_FIRE: r.steps is replaced by the ray's count of steps with an exact test
template <class R, class B>
struct FireProbe {
#ifdef SR_STATS_FIRE
    R& r;
    B& b;
    __device__ FireProbe(R& r_, B& b_) : r(r_), b(b_) { b.fires = 0; }
    __device__ ~FireProbe() { r.steps = b.fires; }
#else
    __device__ FireProbe(R&, B&) {}
#endif
};
template <class B>
__device__ __forceinline__ void probe_fire(B& b) {
#ifdef SR_STATS_FIRE
    b.fires++;
#else
    (void)b;
#endif
}
// phase 1 of a budget event (SR_PROF: events, events spending slot 0 alone,
// lanes spending slot 0)
template <class B>
__device__ __forceinline__ void probe_event_phase1(B& bs, float T, float e0, uint32_t forced, uint32_t spent) {
#ifdef SR_PROF
    const unsigned long long b0 = __ballot(!(T < e0) || (forced & 1u));
    if (SR_LEAD()) {
        bs.prof[16] += 1;
        bs.prof[17] += spent == 1u;
        bs.prof[18] += __popcll(b0);
    }
#else
    (void)bs, (void)T, (void)e0, (void)forced, (void)spent;
#endif
}

// A budget event of the step loop at step i: its interval since the wave's
// previous one, its triggering lanes, and the per-build detail counters
// (tools/stats_frame.py --stephist / --near / --trig / --xcyl, stats_bh.py,
// stats_dir.py). event: this lane triggered it; vb, q0: its ball test and
// ball; bhx: it left the black hole's u window; reseeded, ahead, any_cm: as
// in integrate().
template <class B, class R>
__device__ __forceinline__ void probe_event(const sr_dev_scene* __restrict__ sc, const B& bs, R& r, LoopProbe& lp,
                                            int i, bool event, float vb, float q0, bool bhx, bool reseeded,
                                            float ahead, bool any_cm) {
#ifdef SR_STATS
    r.ev++;
    {  // steps since the wave's previous event, lanes that triggered it (tools/stats_frame.py)
        const int iv = i - lp.last_ev;
        lp.last_ev = i;
        SR_STAT(32 + (iv <= 1 ? 0 : iv <= 3 ? 1 : iv <= 7 ? 2 : iv <= 15 ? 3 : iv <= 63 ? 4 : 5), 1);
        const int nl = __popcll(__ballot(event));
        SR_STAT(38 + (nl <= 1 ? 0 : nl <= 3 ? 1 : nl <= 7 ? 2 : nl <= 15 ? 3 : nl <= 31 ? 4 : 5), 1);
#if defined(SR_STATS_STEPHIST)  // measurement only (tools/stats_frame.py --stephist): events by step
        {
            // events (44 + b) and their triggering lanes (50 + b) by the step
            // index's bucket b: < 25, < 100, < 300, < 700, < 1200, the rest
            const int bk = i < 25 ? 0 : i < 100 ? 1 : i < 300 ? 2 : i < 700 ? 3 : i < 1200 ? 4 : 5;
            SR_STAT(44 + bk, 1);
            SR_STAT(50 + bk, nl);
        }
#elif defined(SR_STATS_NEAR)
        // measurement only (tools/stats_frame.py --near): back-to-back events
        {
            // slots some lane has spent at this event (bit j), by interval 1 (44..46:
            // one, two, three or more slots) and longer (47..49); runs of consecutive
            // interval-1 events, recorded when a longer interval ends one (50..54:
            // 1, 2-3, 4-7, 8-15, 16+); interval-1 events spending one slot, by slot (55..61)
            const float Tt = bs.T();
            uint32_t sm = 0;
            for (int j = 0; j < 7; j++) {
                const float ej = j <= sc->num_budget ? bs.ld(j) : INFINITY;
                if (__ballot(!(Tt < ej))) sm |= 1u << j;
            }
            const int ns = __popc(sm);
            SR_STAT((iv <= 1 ? 44 : 47) + (ns <= 1 ? 0 : ns == 2 ? 1 : 2), 1);
            if (iv <= 1) {
                lp.near_run++;
                if (ns == 1) SR_STAT(55 + __builtin_ctz(sm), 1);
            } else if (lp.near_run > 0) {
                SR_STAT(50 + (lp.near_run <= 1 ? 0 : lp.near_run <= 3 ? 1 : lp.near_run <= 7 ? 2 : lp.near_run <= 15 ? 3 : 4), 1);
                lp.near_run = 0;
            }
        }
#elif defined(SR_STATS_TRIG)  // measurement only (tools/stats_frame.py --trig): who spends which slot
        {
            // lanes whose own budget of slot j ran out (44 + j: orbiting the
            // photon sphere, 51 + j: the others) and events that re-anchor
            // slot j by the look-ahead alone (58 + j)
            const bool ring = r.u > 0.5f && r.u < 0.95f && fabsf(r.du) < 0.15f;
            const float Tt = bs.T();
            for (int j = 0; j < 7; j++) {
                const float ej = j <= sc->num_budget ? bs.ld(j) : INFINITY;
                const bool own = !(Tt < ej);
                SR_STAT(44 + j, __popcll(__ballot(own && ring)));
                SR_STAT(51 + j, __popcll(__ballot(own && !ring)));
                if (j < 6 && __ballot(!(Tt + ahead < ej)) && !__ballot(own)) SR_STAT(58 + j, 1);
            }
        }
#elif defined(SR_STATS_XCYL)  // measurement only (tools/stats_frame.py --xcyl): the cylinder's spends by plane distance
        if (sc->budget_cyl_mask) {
            // lanes spending the first budgeted cylinder (44), of them those whose orbital
            // plane is farther than br + d from its bounding centre, d = 0.25, 1, 2, 4
            // (45..48); events spending it (49), spending it alone (54), and alone with
            // only such lanes (50..53)
            const int jc = __builtin_ctz((uint32_t)sc->budget_cyl_mask) + 1;
            const sr_dev_slot& sl = sc->slots[jc - 1];
            const float Tt = bs.T();
            uint32_t sm = 0;
            for (int j = 0; j <= sc->num_budget; j++)
                if (__ballot(!(Tt < bs.ld(j)))) sm |= 1u << j;
            const bool own = !(Tt < bs.ld(jc));
            const f3 n = cross(r.nv, r.tv);
            const float h = fabsf(dot(ld3(sl.bc), n)) * __builtin_amdgcn_rsqf(dot(n, n)) - sl.br;
            const float dd[4] = {0.25f, 1.0f, 2.0f, 4.0f};
            SR_STAT(44, __popcll(__ballot(own)));
            if (__ballot(own)) SR_STAT(49, 1);
            if (sm == (1u << jc)) SR_STAT(54, 1);
            for (int k = 0; k < 4; k++) {
                SR_STAT(45 + k, __popcll(__ballot(own && h > dd[k])));
                if (sm == (1u << jc) && !__ballot(own && !(h > dd[k]))) SR_STAT(50 + k, 1);
            }
        }
#else
        if (!__ballot(!(vb < 0.0f))) SR_STAT(44, 1);  // the black hole's u window alone
        SR_STAT(45, __popcll(__ballot(event && !(q0 < INFINITY))));  // lanes whose ball was empty
        SR_STAT(46, __popcll(__ballot(bhx)));
        SR_STAT(47, nl);
        if (iv <= 1) {
            SR_STAT(48, nl >= 32);
            SR_STAT(49, __popcll(__ballot(event && !(q0 < INFINITY))));
            SR_STAT(50, nl);
            SR_STAT(51, __popcll(__ballot(event && reseeded)));
            SR_STAT(52, __popcll(__ballot(event && bs.m() < 0.05f)));
            SR_STAT(53, any_cm);
            {  // the slot holding the smallest budget of each triggering lane
                int jm = 0;
                float em = bs.E[0];
                for (int j = 1; j <= sc->num_budget; j++) {
                    const float v = bs.ld(j);
                    if (v < em) { em = v; jm = j; }
                }
                for (int j = 0; j <= 8; j++) SR_STAT(55 + j, __popcll(__ballot(event && jm == j && em < 0.05f)));
            }
        }
        SR_STAT(54, any_cm);
#endif
    }
#endif
#ifdef SR_STATS_BH  // the black hole's triggering lanes by orbit state (tools/stats_bh.py)
    {
        const bool h0 = !(bs.T() < bs.E[0]);
        const bool ring = r.u <= 0.9f && r.u > 0.55f && fabsf(r.du) < 0.1f;
        SR_STAT(23, __popcll(__ballot(h0 && r.u > 1.0f)));
        SR_STAT(24, __popcll(__ballot(h0 && r.u <= 1.0f && r.u > 0.9f)));
        SR_STAT(25, __popcll(__ballot(h0 && ring)));
        SR_STAT(26, __popcll(__ballot(h0 && r.u <= 0.9f && !ring && r.du > 0.0f)));
        SR_STAT(27, __popcll(__ballot(h0 && r.u <= 0.9f && !ring && !(r.du > 0.0f))));
        SR_STAT(28, __popcll(__ballot(event)));
        SR_STAT(29, __popcll(__ballot(h0)));
        SR_STAT(30, __ballot(h0) != 0ull);
        SR_STAT(31, __popcll(__ballot(1)));
    }
#endif
#ifdef SR_STATS_DIR  // object triggers by the lane's radial direction (tools/stats_dir.py)
    {
        const bool outw = r.du < 0.0f && r.u < 0.6f;
        const bool inc = r.du > 0.0f;
        bool any = false;
#pragma unroll
        for (int j = 1; j <= 6; j++) {
            const bool h = !(bs.T() < bs.ld(j));
            any |= h;
            if (j == 3 || j == 5) {  // the default scene's accretion disk and rectangle
                const int b = j == 3 ? 23 : 26;
                SR_STAT(b, __popcll(__ballot(h && outw)));
                SR_STAT(b + 1, __popcll(__ballot(h && inc)));
                SR_STAT(b + 2, __popcll(__ballot(h && !outw && !inc)));
            }
        }
        SR_STAT(29, __popcll(__ballot(any && outw)));
        SR_STAT(30, __popcll(__ballot(any && inc)));
        SR_STAT(31, __popcll(__ballot(any)));
    }
#endif
    (void)sc, (void)bs, (void)r, (void)lp, (void)i, (void)event, (void)vb, (void)q0, (void)bhx, (void)reseeded;
    (void)ahead, (void)any_cm;
}

// ---- per wave (sr_integrate_kernel) --------------------------------------
#ifdef SR_PROF
// the wave's section accumulators (one row per wave of a workgroup of up to 256 threads)
__device__ __forceinline__ unsigned* probe_prof_row() {
    __shared__ unsigned prof_lds[4][SR_PROF_N];
    return prof_lds[threadIdx.x >> 6];
}
#endif
struct WaveProbe {
#ifdef SR_STATS
    unsigned long long t_start, c_start, evmat;
    int rcv[SR_STATS_SLOTS];
#endif
#ifdef SR_PROF
    unsigned long long t0;
#endif
    __device__ WaveProbe() {
#ifdef SR_STATS
        t_start = __builtin_amdgcn_s_memrealtime();
        c_start = __builtin_amdgcn_s_memtime();  // shader clock: the in-kernel clock (rec[15])
        evmat = 0;
        for (int j = 0; j < SR_STATS_SLOTS; j++) rcv[j] = 0;
#endif
#ifdef SR_PROF
        if ((threadIdx.x & 63) < SR_PROF_N) probe_prof_row()[threadIdx.x & 63] = 0;
        t0 = clock64();
#endif
    }
    // SR_LANE_MASK (tools/lane_mask.py): masked pixels run no ray (status `done`)
    __device__ __forceinline__ int lane_mask(int px, int py, int width, int st, int done) const {
#ifdef SR_LANE_MASK
        if (sr_lane_mask && !sr_lane_mask[(size_t)py * width + px]) return done;
#else
        (void)px, (void)py, (void)width, (void)done;
#endif
        return st;
    }
    template <class R>
    __device__ __forceinline__ void ray_start(R& r) const {
#ifdef SR_PROF
        r.prof = probe_prof_row();
        if (SR_LEAD()) r.prof[23] += (unsigned)(clock64() - t0);
#else
        (void)r;
#endif
    }
    // pixels, logged hits, pixels by status (tools/stats_frame.py; wave sums)
    __device__ __forceinline__ void pixel(int st, int n_logged) const {
#if defined(SR_STATS) && !defined(SR_STATS_BH) && !defined(SR_STATS_DIR)
        SR_STAT(23, __popcll(__ballot(1)));
        SR_STAT(24, __popcll(__ballot(n_logged & 1)) + 2 * __popcll(__ballot(n_logged & 2)) +
                        4 * __popcll(__ballot(n_logged & 4)));
        for (int k = 0; k < 6; k++) SR_STAT(25 + k, __popcll(__ballot(st == k)));
#else
        (void)st, (void)n_logged;
#endif
    }
    template <class R>
    __device__ __forceinline__ void ray_end(const R& r) {
#ifdef SR_STATS
        evmat = ((unsigned long long)r.ev << 32) | (unsigned)r.mat;
        for (int j = 0; j < SR_STATS_SLOTS; j++) rcv[j] = r.rc[j];
#else
        (void)r;
#endif
    }
    // the wave's records: SR_STATS its timeline, longest ray, events and
    // reaches (sr_wave_t), SR_PROF its section cycles (sr_prof); every lane
    __device__ __forceinline__ void finish(int frame, int tiles, int block, int ttid, int steps) const {
#ifdef SR_STATS
        {
            int sm = steps;
            unsigned long long em = evmat;
            for (int off = 32; off > 0; off >>= 1) {
                sm = max(sm, __shfl_xor(sm, off));
                const unsigned long long o = __shfl_xor(em, off);
                em = o > em ? o : em;
            }
            int rcm[SR_STATS_SLOTS];
            for (int j = 0; j < SR_STATS_SLOTS; j++) {
                rcm[j] = rcv[j];
                for (int off = 32; off > 0; off >>= 1) rcm[j] = max(rcm[j], __shfl_xor(rcm[j], off));
            }
            const int w = (frame * tiles + block) * 4 + (ttid >> 6);
            if ((threadIdx.x & 63) == 0 && w < SR_WAVE_LOG) {
                unsigned long long* rec = sr_wave_t + (size_t)SR_WAVE_REC * w;
                rec[0] = t_start;
                rec[1] = __builtin_amdgcn_s_memrealtime();
                rec[2] = (unsigned long long)sm;
                rec[3] = em;
                for (int j = 0; j < SR_STATS_SLOTS; j++) rec[4 + j] = (unsigned long long)rcm[j];
                rec[13] = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
                rec[14] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID (wave, SIMD, CU, SE)
                rec[15] = __builtin_amdgcn_s_memtime() - c_start;     // shader-clock cycles of the wave
            }
        }
#endif
#ifdef SR_PROF
        {
            const int w = block * 4 + (ttid >> 6);
            int sm = steps;
            for (int off = 32; off > 0; off >>= 1) sm = max(sm, __shfl_xor(sm, off));
            if ((threadIdx.x & 63) == 0 && w < (1 << 17)) {
                unsigned long long* rec = sr_prof + (size_t)SR_PROF_N * w;
                const unsigned* row = probe_prof_row();
                for (int k = 0; k < SR_PROF_N; k++) rec[k] = row[k];
                rec[7] = (clock64() - t0) | ((unsigned long long)sm << 48);
            }
        }
#endif
        (void)frame, (void)tiles, (void)block, (void)ttid, (void)steps;
    }
};

// ---- host side: the builds' read-out entry points (tools/*.py) -----------
#ifdef SR_PROF
extern "C" int sr_debug_prof(unsigned long long* out, int n_waves) {
    if (n_waves < 0 || n_waves > (1 << 17)) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sr_prof), SR_PROF_N * (size_t)n_waves * sizeof(unsigned long long)) !=
        hipSuccess)
        return -3;
    return 0;
}
#endif

#ifdef SR_LANE_MASK
extern "C" int sr_debug_set_lane_mask(const uint8_t* dev_mask) {
    return hipMemcpyToSymbol(HIP_SYMBOL(sr_lane_mask), &dev_mask, sizeof dev_mask) == hipSuccess ? 0 : -3;
}
#endif

#ifdef SR_STATS
// Measurement builds only: read (and clear) the kernel's event counters.
extern "C" int sr_debug_stats(unsigned long long* out32) {
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(sr_stats), 32 * sizeof(unsigned long long)) != hipSuccess) return -3;
    unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sr_stats), z, sizeof z) != hipSuccess) return -3;
    return 0;
}
// counters 32..63 (read and cleared): event intervals and triggering lanes
extern "C" int sr_debug_stats_hi(unsigned long long* out32) {
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(sr_stats), 32 * sizeof(unsigned long long), 32 * sizeof(unsigned long long)) !=
        hipSuccess)
        return -3;
    unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sr_stats), z, sizeof z, 32 * sizeof(unsigned long long)) != hipSuccess) return -3;
    return 0;
}
extern "C" int sr_debug_wave_times(unsigned long long* out, int n_waves) {
    if (n_waves < 0 || n_waves > SR_WAVE_LOG) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sr_wave_t), SR_WAVE_REC * (size_t)n_waves * sizeof(unsigned long long)) !=
        hipSuccess)
        return -3;
    return 0;
}
#endif

#endif  // SR_PROBES_H
