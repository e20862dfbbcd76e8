// sr_multi_gpu.cpp — the reference's frame loop (src/main.cpp:303-432: one
// full-screen draw per frame, src/main.cpp:318-319) on the GPUs of one node,
// written against the C-ABI of include/sr/sr.h the way a C++ host would
// drive it: RCCL over xGMI, no Python.
//
//   per node    sr_wave_costs (one frame, root GPU) -> sr_block_costs ->
//               sr_balanced_blocks: equal-length lists of 8-row blocks of
//               about equal cost, one per rank
//   per launch  every GPU: sr_render_block_list (B frames, its list) on one
//               of F slots (context + stream + tile), F launches in flight;
//               ncclGather of the equal-size tiles to the root on the GPU's
//               collective stream once that render is done; root:
//               sr_assemble_blocks (device kernel) -> B frames. A slot's next
//               render waits for the gather that read its tile (events only:
//               the host never waits inside the timed loop)
//
// The pipeline is bench.py's (B = 8 frames per launch, F = 3 launches in
// flight at N = 1): a frame's time is the latency of its longest rays'
// waves (the photon ring), and launches in flight fill the SIMDs those waves
// leave idle. At N = 1 there is nothing to gather: a slot's
// tile is the frame (identity block list).
//
// Two ways to run it:
//   one process, N GPUs     ./sr_multi_gpu --gpus N ...        (ncclCommInitAll)
//   one process per GPU     RANK=r WORLD_SIZE=N LOCAL_RANK=r ./sr_multi_gpu [--id-file F] ...
//                           (ncclCommInitRank; rank 0 writes the unique id to F,
//                           prices the blocks and ncclBroadcasts the lists)
// Textures: raw files (--skybox PATH:W:H with RGB8 rows bottom-up, --array
// PATH:W:H:L with RGBA8 layers, as sr_set_background / sr_set_texture_array
// take them) or procedural stand-ins. --out-raw writes the last frame (RGBA8,
// rows bottom-up) for checking; one JSON line goes to stdout.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <unistd.h>
#include <thread>
#include <vector>

#include "sr/sr.h"

namespace {

#define CHECK_SR(x)                                                                           \
    do {                                                                                      \
        const int rc_ = (x);                                                                  \
        if (rc_ != SR_OK) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, sr_status_string(rc_)); \
            std::exit(2);                                                                     \
        }                                                                                     \
    } while (0)
#define CHECK_HIP(x)                                                                          \
    do {                                                                                      \
        const hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                     \
        }                                                                                     \
    } while (0)
#define CHECK_NCCL(x)                                                                         \
    do {                                                                                      \
        const ncclResult_t r_ = (x);                                                          \
        if (r_ != ncclSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
            std::exit(2);                                                                     \
        }                                                                                     \
    } while (0)

constexpr int kBlockRows = 8;  // one 8x8 wave tile tall

struct Args {
    int gpus = 1, width = 1920, height = 1080, max_steps = 2000, frames = 20, batch = 16, warmup = 32, inflight = 2;
    bool flyby = false;
    bool force_gather = false;  // N = 1 too: price, gather (one rank) and reassemble (tests that path)
    std::string skybox, array, out_raw, id_file;
};

void usage() {
    std::printf(
        "sr_multi_gpu [--gpus N] [--width W] [--height H] [--max-steps N] [--frames K] [--batch B]\n"
        "             [--inflight F] [--warmup W] [--flyby] [--skybox PATH:W:H] [--array PATH:W:H:L]\n"
        "             [--out-raw PATH] [--force-gather]\n"
        "             [--id-file PATH]   (one process per GPU: RANK / WORLD_SIZE / LOCAL_RANK from the env)\n");
}

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; i++) {
        const std::string k = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) {
                usage();
                std::exit(1);
            }
            return argv[++i];
        };
        if (k == "--help" || k == "-h") {
            usage();
            std::exit(0);
        } else if (k == "--gpus") a.gpus = std::atoi(next());
        else if (k == "--width") a.width = std::atoi(next());
        else if (k == "--height") a.height = std::atoi(next());
        else if (k == "--max-steps") a.max_steps = std::atoi(next());
        else if (k == "--frames") a.frames = std::atoi(next());
        else if (k == "--batch") a.batch = std::atoi(next());
        else if (k == "--warmup") a.warmup = std::atoi(next());
        else if (k == "--inflight") a.inflight = std::atoi(next());
        else if (k == "--flyby") a.flyby = true;
        else if (k == "--force-gather") a.force_gather = true;
        else if (k == "--skybox") a.skybox = next();
        else if (k == "--array") a.array = next();
        else if (k == "--out-raw") a.out_raw = next();
        else if (k == "--id-file") a.id_file = next();
        else {
            usage();
            std::exit(1);
        }
    }
    return a;
}

std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> out;
    size_t p = 0;
    for (;;) {
        const size_t q = s.find(':', p);
        out.push_back(s.substr(p, q == std::string::npos ? std::string::npos : q - p));
        if (q == std::string::npos) return out;
        p = q + 1;
    }
}

std::vector<uint8_t> read_file(const std::string& path, size_t bytes) {
    std::ifstream f(path, std::ios::binary);
    std::vector<uint8_t> v(bytes);
    if (!f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes)) {
        std::fprintf(stderr, "cannot read %zu bytes from %s\n", bytes, path.c_str());
        std::exit(1);
    }
    return v;
}

// One launch slot of a GPU: its own context (pixel state, launch order), stream and tile.
struct Slot {
    sr_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    uint8_t* tile = nullptr;      // B frames of per * kBlockRows rows
    uint8_t* stacked = nullptr;   // root, N > 1: the gathered tiles of every rank
    uint8_t* frames = nullptr;    // root, N > 1: the reassembled frames (N = 1: the tile itself)
    hipEvent_t rendered = nullptr;  // the slot's render is done (the collective stream waits for it)
    hipEvent_t released = nullptr;  // the gather that read the tile is done (the slot's next render waits)
};

// One GPU's share of the node: F slots and the stream of its collectives.
struct Device {
    int dev = 0;
    ncclComm_t comm = nullptr;
    hipStream_t cstream = nullptr;  // gathers and reassembly, in launch order (one communicator)
    std::vector<Slot> slots;
    // timed launches: render start / end on the slot's stream, gather (+ reassembly) end
    std::vector<hipEvent_t> r0, r1, g1;
    double render_ms_sum = 0.0, gather_ms_sum = 0.0;
};

void setup_slot(Slot& s, int dev, const Args& a, const sr_scene& scene, size_t tile_bytes) {
    CHECK_HIP(hipSetDevice(dev));
    CHECK_SR(sr_create(&s.ctx, dev));
    CHECK_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    CHECK_HIP(hipMalloc(&s.tile, tile_bytes));
    CHECK_HIP(hipEventCreateWithFlags(&s.rendered, hipEventDisableTiming));
    CHECK_HIP(hipEventCreateWithFlags(&s.released, hipEventDisableTiming));
    sr_ctx* ctx = s.ctx;
    CHECK_SR(sr_set_scene(ctx, &scene));
    if (!a.skybox.empty()) {
        const auto f = split(a.skybox);
        const int w = std::atoi(f.at(1).c_str()), h = std::atoi(f.at(2).c_str());
        const auto px = read_file(f[0], (size_t)w * h * 3);
        CHECK_SR(sr_set_background(ctx, px.data(), w, h, 3));
    } else {  // procedural stand-in: an 8x8-cell checker, 2048x1024 RGB
        const int w = 2048, h = 1024;
        std::vector<uint8_t> px((size_t)w * h * 3);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                uint8_t* p = &px[((size_t)y * w + x) * 3];
                const bool c = ((x >> 7) + (y >> 7)) & 1;
                p[0] = (uint8_t)(c ? 200 : 30);
                p[1] = (uint8_t)(x * 255 / w);
                p[2] = (uint8_t)(y * 255 / h);
            }
        CHECK_SR(sr_set_background(ctx, px.data(), w, h, 3));
    }
    if (!a.array.empty()) {
        const auto f = split(a.array);
        const int w = std::atoi(f.at(1).c_str()), h = std::atoi(f.at(2).c_str()), l = std::atoi(f.at(3).c_str());
        const auto px = read_file(f[0], (size_t)w * h * l * 4);
        CHECK_SR(sr_set_texture_array(ctx, px.data(), w, h, l, 4));
    } else {  // opaque stand-in layers of the reference array's size (1601x1201, two layers)
        const int w = 1601, h = 1201, l = 2;
        std::vector<uint8_t> px((size_t)w * h * l * 4);
        for (size_t i = 0; i < (size_t)w * h * l; i++) {
            px[4 * i] = (uint8_t)(i * 7);
            px[4 * i + 1] = (uint8_t)(i * 13);
            px[4 * i + 2] = (uint8_t)(i * 29);
            px[4 * i + 3] = 255;
        }
        CHECK_SR(sr_set_texture_array(ctx, px.data(), w, h, l, 4));
    }
}

}  // namespace

// One process per GPU: the file through which rank 0 hands the RCCL unique id
// to the other ranks. --id-file, else a name unique to the launch: the
// launcher's run id (TORCHELASTIC_RUN_ID) and rendezvous port (MASTER_PORT),
// so concurrent runs with other ports never share a file; with neither (and
// no --id-file) a multi-process run is refused (plain-env launches
// all shared one name). A file with this launch's name but written before the
// launcher that started this rank (a crashed earlier run on the same port) is
// rejected by its modification time against the parent process's start
// (parent_start), whatever the ranks' own start-up skew; rank 0 removes the
// file once every rank has joined.
static bool id_file_path(const std::string& given, std::string& path) {
    if (!given.empty()) {
        path = given;
        return true;
    }
    const char* run = std::getenv("TORCHELASTIC_RUN_ID");
    const char* port = std::getenv("MASTER_PORT");
    const bool has_run = run && *run && std::strcmp(run, "none") != 0, has_port = port && *port;
    path = "/tmp/sr_multi_gpu";
    if (has_run) path += std::string(".") + run;
    if (has_port) path += std::string(".") + port;
    path += ".ncclid";
    return has_run || has_port;
}

// The start time (seconds since the epoch) of this process's parent - the
// launcher that started every rank of the run - from /proc (field 22 of
// /proc/<ppid>/stat in clock ticks after boot, /proc/stat's btime); -1 when
// unknown (then only the file name separates runs).
static double parent_start() {
    std::ifstream st("/proc/" + std::to_string(::getppid()) + "/stat");
    std::string line;
    if (!std::getline(st, line)) return -1.0;
    const size_t close = line.rfind(')');  // the command name may hold spaces
    if (close == std::string::npos) return -1.0;
    std::istringstream rest(line.substr(close + 2));
    std::string f;
    unsigned long long ticks = 0;
    for (int k = 3; k <= 22 && (rest >> f); k++)
        if (k == 22) ticks = std::strtoull(f.c_str(), nullptr, 10);
    std::ifstream ps("/proc/stat");
    unsigned long long btime = 0;
    while (std::getline(ps, line))
        if (line.compare(0, 6, "btime ") == 0) btime = std::strtoull(line.c_str() + 6, nullptr, 10);
    const long hz = ::sysconf(_SC_CLK_TCK);
    if (!ticks || !btime || hz <= 0) return -1.0;
    return (double)btime + (double)ticks / (double)hz;
}

int main(int argc, char** argv) {
    Args a = parse(argc, argv);
    const char* ws = std::getenv("WORLD_SIZE");
    const bool per_process = ws && std::atoi(ws) > 1;
    const int world = per_process ? std::atoi(ws) : a.gpus;
    const int rank = per_process ? std::atoi(std::getenv("RANK") ? std::getenv("RANK") : "0") : 0;
    const int local = per_process ? std::atoi(std::getenv("LOCAL_RANK") ? std::getenv("LOCAL_RANK") : "0") : 0;
    int ndev = 0;
    CHECK_HIP(hipGetDeviceCount(&ndev));
    if (!per_process && (world < 1 || world > ndev)) {
        std::fprintf(stderr, "--gpus %d: %d device(s) visible\n", world, ndev);
        return 1;
    }
    if (a.batch < 1 || a.batch > 32 || a.frames < 1 || a.inflight < 1 || a.inflight > 8 || a.warmup < 0) {
        std::fprintf(stderr, "--batch must be 1..32, --inflight 1..8, --frames >= 1, --warmup >= 0\n");
        return 1;
    }
    const int W = a.width, H = a.height, B = a.batch, F = a.inflight;
    // warmup of at least one launch per slot: a slot's context learns its launch
    // order from its own first launch, so an unwarmed slot's first timed launch
    // would run in the default order
    a.warmup = std::max(a.warmup, B * F);
    const bool gather = world > 1 || a.force_gather;  // N = 1: the tile is the frame
    const int nb = (H + kBlockRows - 1) / kBlockRows, nc = (W + 7) / 8;
    const int per = (nb + world - 1) / world;
    const size_t row_bytes = (size_t)W * 4, tile_frame = (size_t)per * kBlockRows * row_bytes;
    const size_t tile_bytes = tile_frame * B;

    sr_scene scene;
    sr_default_scene(&scene);  // src/main.cpp:222-268
    if (!a.array.empty()) {
        const auto f = split(a.array);
        scene.max_texture_size[0] = (float)std::atoi(f.at(1).c_str());
        scene.max_texture_size[1] = (float)std::atoi(f.at(2).c_str());
    }
    sr_params params;
    sr_params_default(&params);
    params.max_steps = a.max_steps;
    params.percent_black = -1.0f;  // the benchmark's setting

    // ---- devices and communicators (one per GPU: the gathers run in launch
    // order on each GPU's collective stream) ----
    std::vector<Device> devs(per_process ? 1 : world);
    if (per_process) {
        devs[0].dev = local % ndev;
        ncclUniqueId id;
        std::string path;
        if (!id_file_path(a.id_file, path)) {
            std::fprintf(stderr, "rank %d: WORLD_SIZE > 1 needs --id-file, MASTER_PORT or TORCHELASTIC_RUN_ID "
                                 "(a name no other launch shares)\n", rank);
            return 1;
        }
        if (rank == 0) {
            CHECK_NCCL(ncclGetUniqueId(&id));
            const std::string tmp = path + ".tmp";
            std::ofstream(tmp, std::ios::binary).write(reinterpret_cast<const char*>(&id), sizeof id);
            std::rename(tmp.c_str(), path.c_str());
        } else {
            // a file written before this run's launcher started is a previous
            // run's: never hand its id to ncclCommInitRank (btime is whole
            // seconds, so the launcher's start is known to within 1 s)
            const double launched = parent_start();
            for (int t = 0;; t++) {
                struct stat st;
                if (::stat(path.c_str(), &st) == 0 &&
                    (launched < 0.0 || (double)st.st_mtim.tv_sec + 1e-9 * (double)st.st_mtim.tv_nsec >= launched - 1.0)) {
                    std::ifstream f(path, std::ios::binary);
                    if (f.read(reinterpret_cast<char*>(&id), sizeof id)) break;
                }
                if (t > 6000) {
                    std::fprintf(stderr, "rank %d: no NCCL id of this run in %s\n", rank, path.c_str());
                    return 1;
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            }
        }
        CHECK_HIP(hipSetDevice(devs[0].dev));
        CHECK_NCCL(ncclCommInitRank(&devs[0].comm, world, id, rank));
        // every rank has joined once rank 0's init returns: no later run can read this id
        if (rank == 0) std::remove(path.c_str());
    } else {
        std::vector<ncclComm_t> comms(world);
        std::vector<int> ids(world);
        for (int d = 0; d < world; d++) ids[d] = devs[d].dev = d;
        CHECK_NCCL(ncclCommInitAll(comms.data(), world, ids.data()));
        for (int d = 0; d < world; d++) devs[d].comm = comms[d];
    }
    const bool root = rank == 0;  // devs[0] is the root GPU in the one-process mode
    for (size_t k = 0; k < devs.size(); k++) {
        Device& d = devs[k];
        d.slots.resize(F);
        for (auto& s : d.slots) setup_slot(s, d.dev, a, scene, tile_bytes);
        CHECK_HIP(hipSetDevice(d.dev));
        CHECK_HIP(hipStreamCreateWithFlags(&d.cstream, hipStreamNonBlocking));
    }
    Device& r0 = devs[0];

    // cameras: the app's default, or its H-key flyby (src/main.cpp:404-410)
    const int n_total = a.warmup + a.frames;
    std::vector<sr_camera> cams(n_total);
    for (int f = 0; f < n_total; f++) {
        sr_default_camera(&cams[f]);
        if (a.flyby) CHECK_SR(sr_camera_hyperbolic_trajectory(&cams[f], 30.0f, 10.0f, (f + 0.5f) / n_total));
    }

    // ---- pricing on the root GPU, lists to every rank (N = 1: every block in order) ----
    std::vector<int> lists((size_t)world * per, -1);
    double max_over_mean = 1.0;
    if (!gather) {
        for (int b = 0; b < nb; b++) lists[b] = b;
    } else {
        int32_t* d_costs = nullptr;
        Slot& p0 = r0.slots[0];
        if (root) {
            CHECK_HIP(hipSetDevice(r0.dev));
            CHECK_HIP(hipMalloc(&d_costs, (size_t)nb * nc * 2 * sizeof(int32_t)));
            CHECK_SR(sr_wave_costs(p0.ctx, &cams[0], &params, W, H, d_costs, p0.stream));
            std::vector<int32_t> wc((size_t)nb * nc * 2);
            CHECK_HIP(hipMemcpyAsync(wc.data(), d_costs, wc.size() * sizeof(int32_t), hipMemcpyDeviceToHost, p0.stream));
            CHECK_HIP(hipStreamSynchronize(p0.stream));
            CHECK_HIP(hipFree(d_costs));
            std::vector<double> cost(nb);
            CHECK_SR(sr_block_costs(wc.data(), nb, nc, 8.0, cost.data()));
            int got = 0;
            CHECK_SR(sr_balanced_blocks(cost.data(), nb, world, lists.data(), (int)lists.size(), &got));
            double mx = 0.0, sum = 0.0;
            for (int r = 0; r < world; r++) {
                double l = 0.0;
                for (int s = 0; s < per; s++)
                    if (lists[(size_t)r * per + s] >= 0) l += cost[lists[(size_t)r * per + s]];
                mx = std::max(mx, l);
                sum += l;
            }
            max_over_mean = sum > 0.0 ? mx / (sum / world) : 1.0;
        }
        if (per_process) {  // the root's lists to every rank (one broadcast, int32)
            int* d_l = nullptr;
            CHECK_HIP(hipSetDevice(r0.dev));
            CHECK_HIP(hipMalloc(&d_l, lists.size() * sizeof(int)));
            CHECK_HIP(hipMemcpyAsync(d_l, lists.data(), lists.size() * sizeof(int), hipMemcpyHostToDevice, r0.cstream));
            CHECK_NCCL(ncclBroadcast(d_l, d_l, lists.size(), ncclInt32, 0, r0.comm, r0.cstream));
            CHECK_HIP(hipMemcpyAsync(lists.data(), d_l, lists.size() * sizeof(int), hipMemcpyDeviceToHost, r0.cstream));
            CHECK_HIP(hipStreamSynchronize(r0.cstream));
            CHECK_HIP(hipFree(d_l));
        }
    }

    // root buffers (gather): per slot the gathered tiles and the frames; the lists on the device
    int* d_lists = nullptr;
    if (root && gather) {
        CHECK_HIP(hipSetDevice(r0.dev));
        for (auto& s : r0.slots) {
            CHECK_HIP(hipMalloc(&s.stacked, tile_bytes * world));
            CHECK_HIP(hipMalloc(&s.frames, (size_t)B * H * row_bytes));
        }
        CHECK_HIP(hipMalloc(&d_lists, lists.size() * sizeof(int)));
        CHECK_HIP(hipMemcpy(d_lists, lists.data(), lists.size() * sizeof(int), hipMemcpyHostToDevice));
    }

    // launch j: frames [first, first + n) on slot j % F of every GPU, then
    // (N > 1) the gather and the reassembly on the collective streams. Events
    // order it: no host wait. t >= 0: the timed launch's index.
    int launches = 0;
    auto launch = [&](int first, int n, int t) {
        const int k = launches % F;
        const bool reuse = launches >= F;
        launches++;
        for (size_t i = 0; i < devs.size(); i++) {
            Device& d = devs[i];
            Slot& s = d.slots[k];
            const int r = per_process ? rank : (int)i;
            CHECK_HIP(hipSetDevice(d.dev));
            if (reuse && gather) CHECK_HIP(hipStreamWaitEvent(s.stream, s.released, 0));  // its tile was gathered
            if (t >= 0) CHECK_HIP(hipEventRecord(d.r0[t], s.stream));
            CHECK_SR(sr_render_block_list(s.ctx, &cams[first], n, &params, W, H, kBlockRows, &lists[(size_t)r * per],
                                          per, s.tile, row_bytes, tile_frame, s.stream));
            if (t >= 0) CHECK_HIP(hipEventRecord(d.r1[t], s.stream));
            if (gather) {
                CHECK_HIP(hipEventRecord(s.rendered, s.stream));
                CHECK_HIP(hipStreamWaitEvent(d.cstream, s.rendered, 0));
            }
        }
        if (gather) {
            // equal-size tiles to the root over xGMI (each peer on its own link)
            CHECK_NCCL(ncclGroupStart());
            for (size_t i = 0; i < devs.size(); i++) {
                Device& d = devs[i];
                Slot& s = d.slots[k];
                const bool is_root = per_process ? root : i == 0;
                CHECK_NCCL(ncclGather(s.tile, is_root ? r0.slots[k].stacked : nullptr, tile_bytes, ncclUint8, 0, d.comm,
                                      d.cstream));
            }
            CHECK_NCCL(ncclGroupEnd());
            if (root) {
                Slot& s = r0.slots[k];
                CHECK_HIP(hipSetDevice(r0.dev));
                CHECK_SR(sr_assemble_blocks(s.stacked, tile_bytes, tile_frame, d_lists, world, per, H, kBlockRows,
                                            row_bytes, s.frames, (size_t)H * row_bytes, n, 1, r0.cstream));
            }
            for (auto& d : devs) {
                CHECK_HIP(hipSetDevice(d.dev));
                CHECK_HIP(hipEventRecord(d.slots[k].released, d.cstream));
                if (t >= 0) CHECK_HIP(hipEventRecord(d.g1[t], d.cstream));
            }
        } else if (t >= 0) {
            CHECK_HIP(hipEventRecord(r0.g1[t], r0.slots[k].stream));
        }
        return k;
    };
    auto sync_all = [&]() {
        for (auto& d : devs) {
            CHECK_HIP(hipSetDevice(d.dev));
            for (auto& s : d.slots) CHECK_HIP(hipStreamSynchronize(s.stream));
            CHECK_HIP(hipStreamSynchronize(d.cstream));
        }
    };
    const int n_timed = (a.frames + B - 1) / B;
    for (auto& d : devs) {
        CHECK_HIP(hipSetDevice(d.dev));
        for (auto* v : {&d.r0, &d.r1, &d.g1}) {
            v->resize(n_timed);
            for (auto& e : *v) CHECK_HIP(hipEventCreate(&e));
        }
    }
    // warmup: every slot's context learns the launch order of its tiles
    for (int f = 0; f < a.warmup; f += B) launch(f, std::min(B, a.warmup - f), -1);
    sync_all();
    const auto t0 = std::chrono::steady_clock::now();
    int last_n = 0, last_k = 0, t = 0;
    for (int f = 0; f < a.frames; f += B, t++) {
        last_n = std::min(B, a.frames - f);
        last_k = launch(a.warmup + f, last_n, t);
    }
    sync_all();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // device times of the timed launches (read after the loop): the launches
    // overlap, so render_ms sums to more than the wall time
    for (auto& d : devs) {
        double rm = 0.0, gm = 0.0;
        for (int i = 0; i < n_timed; i++) {
            float x = 0.f, y = 0.f;
            CHECK_HIP(hipEventElapsedTime(&x, d.r0[i], d.r1[i]));
            CHECK_HIP(hipEventElapsedTime(&y, d.r1[i], d.g1[i]));
            rm += x;
            gm += y;
        }
        d.render_ms_sum = rm;
        d.gather_ms_sum = gm;
    }

    if (root && !a.out_raw.empty()) {  // the run's last frame
        std::vector<uint8_t> h((size_t)H * row_bytes);
        const Slot& s = r0.slots[last_k];
        const uint8_t* src = gather ? s.frames + (size_t)(last_n - 1) * H * row_bytes
                                       : s.tile + (size_t)(last_n - 1) * tile_frame;
        CHECK_HIP(hipSetDevice(r0.dev));
        CHECK_HIP(hipMemcpy(h.data(), src, h.size(), hipMemcpyDeviceToHost));
        std::ofstream(a.out_raw, std::ios::binary).write(reinterpret_cast<const char*>(h.data()), (std::streamsize)h.size());
    }
    if (root) {
        std::printf("{\"tool\": \"sr_multi_gpu\", \"mode\": \"%s\", \"world_size\": %d, \"width\": %d, \"height\": %d, "
                    "\"max_steps\": %d, \"frames\": %d, \"warmup\": %d, \"frames_per_launch\": %d, "
                    "\"launches_in_flight\": %d, \"camera\": \"%s\", "
                    "\"value\": %.3f, \"unit\": \"Mpixels/s\", \"ms_per_frame\": %.4f, \"balance_max_over_mean\": %.4f, "
                    "\"timing\": \"wall clock around the timed launches, streams synchronised on both sides\", "
                    "\"collective\": \"%s\", \"ranks\": [",
                    per_process ? "process per GPU (ncclCommInitRank)" : "one process (ncclCommInitAll)", world, W, H,
                    a.max_steps, a.frames, a.warmup, B, F, a.flyby ? "flyby" : "static",
                    (double)W * H * a.frames / sec / 1e6, sec * 1e3 / a.frames, max_over_mean,
                    gather ? "ncclGather of equal-size tiles on each GPU's collective stream"
                              : "none (one GPU: the tile is the frame)");
        for (size_t k = 0; k < devs.size(); k++)
            std::printf("%s{\"device\": %d, \"render_ms_per_launch\": %.4f, \"render_ms_per_frame\": %.4f, "
                        "\"gather_ms_per_frame\": %.4f}",
                        k ? ", " : "", devs[k].dev, devs[k].render_ms_sum / n_timed, devs[k].render_ms_sum / a.frames,
                        devs[k].gather_ms_sum / a.frames);
        std::printf("]}\n");
    }
    for (auto& d : devs) {
        CHECK_HIP(hipSetDevice(d.dev));
        for (auto& s : d.slots) {
            sr_destroy(s.ctx);
            (void)hipFree(s.tile);
            if (s.stacked) (void)hipFree(s.stacked);
            if (s.frames) (void)hipFree(s.frames);
            (void)hipStreamDestroy(s.stream);
            (void)hipEventDestroy(s.rendered);
            (void)hipEventDestroy(s.released);
        }
        for (auto* v : {&d.r0, &d.r1, &d.g1})
            for (auto& e : *v) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(d.cstream);
        (void)ncclCommDestroy(d.comm);
    }
    if (d_lists) {
        CHECK_HIP(hipSetDevice(r0.dev));
        (void)hipFree(d_lists);
    }
    return 0;
}
