// partition.cpp — the multi-GPU frame partition behind the C-ABI (sr.h
// sr_block_costs / sr_balanced_blocks / sr_assemble_blocks, host side).
//
// Not in the reference: its frame is one full-screen draw on one GPU
// (src/main.cpp:318-319). Here a frame's rows are cut into 8-row blocks, each
// rank of a node renders an equal-length list of blocks of about equal cost
// (sr_render_block_list) and the root reassembles the gathered tiles (SURVEY
// §8e). Pricing comes from one per-wave cost map (sr_wave_costs): a wave
// runs until its longest ray is done, and a budget event costs about
// EVENT_STEPS wave-steps. The dealing rule is the one of
// schwarzschild-raytracer_amd/dist.py balanced_blocks, operation for
// operation in binary64, so a C++ caller and the Python bench derive the same
// lists from the same costs (tests/test_partition.py).
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "sr/sr.h"

extern "C" {

int sr_block_costs(const int32_t* wave_cost, int n_blocks, int waves_per_block, double event_steps,
                   double* out_cost) {
    if (!wave_cost || !out_cost || n_blocks < 0 || waves_per_block < 0) return SR_E_INVALID;
    for (int b = 0; b < n_blocks; b++) {
        // numpy's sum over a row of float64 values, left to right from the first
        double s = 0.0;
        for (int c = 0; c < waves_per_block; c++) {
            const int32_t* w = wave_cost + ((size_t)b * waves_per_block + c) * 2;
            const double v = (double)w[0] + event_steps * (double)w[1];
            s = c == 0 ? v : s + v;
        }
        out_cost[b] = s;
    }
    return SR_OK;
}

int sr_balanced_blocks(const double* cost, int n_blocks, int world, int* out_lists, int max_entries, int* out_per) {
    if (!cost || !out_lists || !out_per || n_blocks < 0 || world <= 0) return SR_E_INVALID;
    const int per = (n_blocks + world - 1) / world;
    *out_per = per;
    if ((long long)per * world > max_entries) return SR_E_CAPACITY;
    auto c_of = [&](int b) { return b >= 0 ? cost[b] : 0.0; };
    // blocks by descending cost (ties: lower index), each to the rank with
    // the least load among those with room (ties: lower rank)
    std::vector<int> order(n_blocks);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    std::vector<std::vector<int>> lists(world);
    std::vector<double> load(world, 0.0);
    for (int b : order) {
        int r = -1;
        for (int k = 0; k < world; k++) {
            if ((int)lists[k].size() >= per) continue;
            if (r < 0 || load[k] < load[r]) r = k;
        }
        lists[r].push_back(b);
        load[r] += cost[b];
    }
    for (auto& l : lists) l.resize(per, -1);
    // pairwise swaps out of the most loaded rank while one lowers the pair's maximum
    for (int it = 0; it < 4 * n_blocks; it++) {
        int hi = 0;
        for (int k = 1; k < world; k++)
            if (load[k] > load[hi]) hi = k;
        bool found = false;
        double bm = 0.0, bd = 0.0;
        int br = 0, bi = 0, bj = 0;
        for (int r = 0; r < world; r++) {
            if (r == hi) continue;
            for (int i = 0; i < per; i++) {
                for (int j = 0; j < per; j++) {
                    const double d = c_of(lists[hi][i]) - c_of(lists[r][j]);
                    if (d <= 0.0) continue;
                    const double m = std::max(load[hi] - d, load[r] + d);
                    if (m < load[hi] - 1e-9 && (!found || m < bm)) {
                        found = true;
                        bm = m;
                        br = r;
                        bi = i;
                        bj = j;
                        bd = d;
                    }
                }
            }
        }
        if (!found) break;
        std::swap(lists[hi][bi], lists[br][bj]);
        load[hi] -= bd;
        load[br] += bd;
    }
    // block-cyclic lists when they are at least as even
    double cyc_max = 0.0;
    for (int k = 0; k < world; k++) {
        double s = 0.0;
        for (int b = k; b < n_blocks; b += world) s += cost[b];
        cyc_max = k == 0 ? s : std::max(cyc_max, s);
    }
    const double lmax = *std::max_element(load.begin(), load.end());
    for (int k = 0; k < world; k++) {
        int* o = out_lists + (size_t)k * per;
        if (cyc_max <= lmax) {
            int s = 0;
            for (int b = k; b < n_blocks; b += world) o[s++] = b;
            for (; s < per; s++) o[s] = -1;
        } else {
            std::vector<int> l;
            for (int b : lists[k])
                if (b >= 0) l.push_back(b);
            std::sort(l.begin(), l.end());
            int s = 0;
            for (int b : l) o[s++] = b;
            for (; s < per; s++) o[s] = -1;
        }
    }
    return SR_OK;
}

// Host reassembly (on_device == 0); the device path is sr_assemble_blocks_device (kernels/assemble.hip).
int sr_assemble_blocks_host(const uint8_t* stacked, size_t rank_stride, size_t in_frame_stride, const int* lists,
                            int world, int per, int height, int block_rows, size_t row_bytes, uint8_t* out,
                            size_t out_frame_stride, int n_frames) {
    for (int f = 0; f < n_frames; f++) {
        for (int r = 0; r < world; r++) {
            for (int s = 0; s < per; s++) {
                const int b = lists[(size_t)r * per + s];
                if (b < 0) continue;
                for (int j = 0; j < block_rows; j++) {
                    const int y = b * block_rows + j;
                    if (y >= height) break;
                    std::memcpy(out + (size_t)f * out_frame_stride + (size_t)y * row_bytes,
                                stacked + (size_t)r * rank_stride + (size_t)f * in_frame_stride +
                                    ((size_t)s * block_rows + j) * row_bytes,
                                row_bytes);
                }
            }
        }
    }
    return SR_OK;
}

}  // extern "C"
