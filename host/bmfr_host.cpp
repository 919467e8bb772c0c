// bmfr_host.cpp -- the reference's host program (bmfr.cpp: tasks() / main())
// on libbmfr's C ABI (include/bmfr.h) and HIP instead of OpenCL.
//
// Same #define surface and file conventions as bmfr.cpp:32-118 (overridable
// on the command line), same frame loop (bmfr.cpp:417-485) and profiling
// report (bmfr.cpp:488-517), same outputs (outputs/outputNN.png,
// bmfr.cpp:519-553).  Differences, all on the host side:
//   * EXR / PNG I/O through host/image_io.cpp (OpenImageIO is not in this
//     toolchain); camera_matrices.h is parsed at run time (--camera) instead
//     of being #included at build time;
//   * uploads of frame f+1 overlap frame f on a copy stream (SURVEY 8f4;
//     the reference uploads synchronously, bmfr.cpp:420-427);
//   * --synthetic runs the built-in synthetic scene (no dataset needed),
//     --write-synthetic writes it as a dataset (EXRs + camera_matrices.h),
//     --psnr compares the outputs with reference images.
#include <hip/hip_runtime.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "bmfr.h"
#include "image_io.h"

// ### bmfr.cpp:39-91 defaults ###
#define IMAGE_WIDTH 1280
#define IMAGE_HEIGHT 720
#define FRAME_COUNT 60
#define INPUT_DATA_PATH "../data/frames"
#define NOISY_FILE_NAME "/color"
#define NORMAL_FILE_NAME "/shading_normal"
#define POSITION_FILE_NAME "/world_position"
#define ALBEDO_FILE_NAME "/albedo"
#define OUTPUT_FILE_NAME "outputs/output"
#define NOISE_AMOUNT 1e-2
#define BLEND_ALPHA 0.2f
#define SECOND_BLEND_ALPHA 0.1f
#define TAA_BLEND_ALPHA 0.2f
#define NOT_SCALED_FEATURE_BUFFERS \
    "1.f,"                         \
    "normal.x,"                    \
    "normal.y,"                    \
    "normal.z,"
#define SCALED_FEATURE_BUFFERS             \
    "world_position.x,"                    \
    "world_position.y,"                    \
    "world_position.z,"                    \
    "world_position.x*world_position.x,"   \
    "world_position.y*world_position.y,"   \
    "world_position.z*world_position.z"
#define USE_HALF_PRECISION_IN_TMP_DATA 1

namespace {

struct Options {
    int width = IMAGE_WIDTH, height = IMAGE_HEIGHT, frames = FRAME_COUNT;
    std::string input = INPUT_DATA_PATH, camera, output = OUTPUT_FILE_NAME, psnr, write_synthetic;
    std::string not_scaled = NOT_SCALED_FEATURE_BUFFERS, scaled = SCALED_FEATURE_BUFFERS;
    bool synthetic = false, exr = false, pipelined = true, save = true;
    int half_tmp = USE_HALF_PRECISION_IN_TMP_DATA;
    int device = 0;
    unsigned seed = 0x424D4652;
    // --tile-grid TXxTY: the frame sharded into tiles, one libbmfr context per
    // tile, the halo exchanged by bmfr_exchange_run_all (RCCL between devices
    // with --gpus N = tiles, device copies when every tile is on one GPU)
    int tiles_x = 0, tiles_y = 0, tile_halo = 64, gpus = 1;
    int fast_fit = 0;
};

void usage() {
    std::printf(
        "bmfr_host [options]   (defaults: bmfr.cpp's #defines)\n"
        "  --input DIR            dataset folder: colorNN.exr, shading_normalNN.exr, world_positionNN.exr,\n"
        "                         albedoNN.exr, camera_matrices.h (default " INPUT_DATA_PATH ")\n"
        "  --camera FILE          camera_matrices.h (default DIR/camera_matrices.h)\n"
        "  --synthetic            built-in synthetic scene instead of files\n"
        "  --write-synthetic DIR  write the synthetic scene as a dataset and exit\n"
        "  --width W --height H --frames N\n"
        "  --output PREFIX        output file prefix (default " OUTPUT_FILE_NAME ")\n"
        "  --exr                  write float EXR outputs instead of PNG\n"
        "  --no-save              do not write outputs\n"
        "  --psnr PREFIX          PSNR of each output vs PREFIXNN.exr (tone-mapped like the output)\n"
        "  --features-not-scaled S --features-scaled S   feature lists as in bmfr.cpp:65-77\n"
        "  --half-tmp 0|1         USE_HALF_PRECISION_IN_TMP_DATA\n"
        "  --no-pipeline          synchronous uploads (as bmfr.cpp)\n"
        "  --device I\n"
        "  --tile-grid TXxTY      shard each frame into TX x TY tiles (one context per tile, halo exchange\n"
        "                         between frames: bmfr_exchange_run_all)\n"
        "  --tile-halo PX         tile halo in pixels (default 64; >= 34 + the scene's motion per frame)\n"
        "  --gpus N               tiles on N GPUs from --device on (N = 1: all on one GPU, device copies;\n"
        "                         N = tiles: one GPU per tile, RCCL)\n"
        "  --fast-fit             bmfr_config.fast_fit = 1\n");
}

bool parse_args(int argc, char** argv, Options& o) {
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&](const char* what) -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "%s needs %s\n", a.c_str(), what);
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--input") o.input = next("a folder");
        else if (a == "--camera") o.camera = next("a file");
        else if (a == "--synthetic") o.synthetic = true;
        else if (a == "--write-synthetic") o.write_synthetic = next("a folder");
        else if (a == "--width") o.width = std::atoi(next("pixels"));
        else if (a == "--height") o.height = std::atoi(next("pixels"));
        else if (a == "--frames") o.frames = std::atoi(next("a count"));
        else if (a == "--output") o.output = next("a prefix");
        else if (a == "--exr") o.exr = true;
        else if (a == "--no-save") o.save = false;
        else if (a == "--psnr") o.psnr = next("a prefix");
        else if (a == "--features-not-scaled") o.not_scaled = next("a list");
        else if (a == "--features-scaled") o.scaled = next("a list");
        else if (a == "--half-tmp") o.half_tmp = std::atoi(next("0 or 1"));
        else if (a == "--no-pipeline") o.pipelined = false;
        else if (a == "--device") o.device = std::atoi(next("an index"));
        else if (a == "--seed") o.seed = (unsigned)std::strtoul(next("a number"), nullptr, 0);
        else if (a == "--tile-grid") {
            const char* g = next("TXxTY");
            if (std::sscanf(g, "%dx%d", &o.tiles_x, &o.tiles_y) != 2 || o.tiles_x < 1 || o.tiles_y < 1) {
                std::fprintf(stderr, "--tile-grid wants TXxTY, got %s\n", g);
                return false;
            }
        } else if (a == "--tile-halo") o.tile_halo = std::atoi(next("pixels"));
        else if (a == "--gpus") o.gpus = std::atoi(next("a count"));
        else if (a == "--fast-fit") o.fast_fit = 1;
        else if (a == "-h" || a == "--help") {
            usage();
            std::exit(0);
        } else {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            usage();
            return false;
        }
    }
    if (o.camera.empty()) o.camera = o.input + "/camera_matrices.h";
    return true;
}

// FEATURE_BUFFERS strings (bmfr.cpp:65-77) -> bmfr_feature codes.  The
// reference pastes them into the kernels as C expressions; these are the
// monomials of normal / world_position it can name.
bool parse_features(const std::string& list, std::vector<int>& out) {
    static const struct {
        const char* expr;
        int code;
    } kMap[] = {{"1.f", BMFR_FEATURE_ONE},
                {"normal.x", BMFR_FEATURE_NORMAL_X},
                {"normal.y", BMFR_FEATURE_NORMAL_Y},
                {"normal.z", BMFR_FEATURE_NORMAL_Z},
                {"world_position.x", BMFR_FEATURE_POSITION_X},
                {"world_position.y", BMFR_FEATURE_POSITION_Y},
                {"world_position.z", BMFR_FEATURE_POSITION_Z},
                {"world_position.x*world_position.x", BMFR_FEATURE_POSITION_X2},
                {"world_position.y*world_position.y", BMFR_FEATURE_POSITION_Y2},
                {"world_position.z*world_position.z", BMFR_FEATURE_POSITION_Z2},
                {"world_position.x*world_position.x*world_position.x", BMFR_FEATURE_POSITION_X3},
                {"world_position.y*world_position.y*world_position.y", BMFR_FEATURE_POSITION_Y3},
                {"world_position.z*world_position.z*world_position.z", BMFR_FEATURE_POSITION_Z3}};
    std::stringstream ss(list);
    std::string item;
    while (std::getline(ss, item, ',')) {
        item.erase(std::remove_if(item.begin(), item.end(), ::isspace), item.end());
        if (item.empty()) continue;
        bool found = false;
        for (const auto& m : kMap)
            if (item == m.expr) {
                out.push_back(m.code);
                found = true;
            }
        if (!found) {
            std::fprintf(stderr, "unsupported feature expression '%s'\n", item.c_str());
            return false;
        }
    }
    return true;
}

// camera_matrices.h of the BMFR dataset: float arrays camera_matrices[F][4][4]
// and pixel_offsets[F][2], scalars position_limit_squared and
// normal_limit_squared (bmfr.cpp:44-47, 226-227, 440-444).
struct Camera {
    std::vector<float> matrices, offsets;
    double position_limit_squared = 0.01, normal_limit_squared = 0.1;
};

std::vector<double> numbers_after(const std::string& text, const std::string& name, size_t& pos) {
    std::vector<double> v;
    pos = text.find(name);
    if (pos == std::string::npos) return v;
    size_t p = text.find('=', pos);
    if (p == std::string::npos) return v;
    ++p;
    int depth = 0;
    bool in_braces = false;
    while (p < text.size()) {
        const char c = text[p];
        if (c == '{') {
            ++depth;
            in_braces = true;
            ++p;
        } else if (c == '}') {
            if (--depth <= 0) break;
            ++p;
        } else if (c == ';' && depth == 0) {
            break;
        } else if (std::isdigit((unsigned char)c) || c == '-' || c == '+' || c == '.') {
            char* end = nullptr;
            const double d = std::strtod(text.c_str() + p, &end);
            if (end == text.c_str() + p) {
                ++p;
                continue;
            }
            v.push_back(d);
            p = end - text.c_str();
            while (p < text.size() && (text[p] == 'f' || text[p] == 'F')) ++p;
            if (!in_braces) break;
        } else {
            ++p;
        }
    }
    return v;
}

bool load_camera(const std::string& path, int frames, Camera& cam) {
    std::ifstream f(path);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string t = ss.str();
    size_t pos;
    std::vector<double> m = numbers_after(t, "camera_matrices", pos);
    std::vector<double> o = numbers_after(t, "pixel_offsets", pos);
    std::vector<double> pl = numbers_after(t, "position_limit_squared", pos);
    std::vector<double> nl = numbers_after(t, "normal_limit_squared", pos);
    if (m.size() < (size_t)frames * 16 || o.size() < (size_t)frames * 2 || pl.empty() || nl.empty()) return false;
    cam.matrices.assign(m.begin(), m.begin() + (size_t)frames * 16);
    cam.offsets.assign(o.begin(), o.begin() + (size_t)frames * 2);
    cam.position_limit_squared = pl[0];
    cam.normal_limit_squared = nl[0];
    return true;
}

bool write_camera(const std::string& path, int frames, const Camera& cam) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return false;
    std::fprintf(f, "// Synthetic sequence written by bmfr_host --write-synthetic\n");
    std::fprintf(f, "const float position_limit_squared = %.9g;\nconst float normal_limit_squared = %.9g;\n",
                 cam.position_limit_squared, cam.normal_limit_squared);
    std::fprintf(f, "static const float camera_matrices[%d][4][4] = {\n", frames);
    for (int i = 0; i < frames; ++i) {
        std::fprintf(f, "  {");
        for (int r = 0; r < 4; ++r) {
            std::fprintf(f, "{");
            for (int c = 0; c < 4; ++c) std::fprintf(f, "%.9g%s", cam.matrices[i * 16 + r * 4 + c], c < 3 ? ", " : "");
            std::fprintf(f, "}%s", r < 3 ? ", " : "");
        }
        std::fprintf(f, "}%s\n", i + 1 < frames ? "," : "");
    }
    std::fprintf(f, "};\nstatic const float pixel_offsets[%d][2] = {\n", frames);
    for (int i = 0; i < frames; ++i)
        std::fprintf(f, "  {%.9g, %.9g}%s\n", cam.offsets[2 * i], cam.offsets[2 * i + 1], i + 1 < frames ? "," : "");
    std::fprintf(f, "};\n");
    return std::fclose(f) == 0;
}

std::string frame_file(const std::string& prefix, int frame, const char* ext) {
    return prefix + std::to_string(frame) + ext;
}

#define HIP_CHECK(x)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

#define BMFR_CHECK(x)                                                                       \
    do {                                                                                    \
        bmfr_status s_ = (x);                                                               \
        if (s_ != BMFR_OK) {                                                                \
            std::fprintf(stderr, "%s failed: %s (hip error %d)\n", #x, bmfr_status_string(s_), \
                         bmfr_last_hip_error());                                            \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

double tonemap(float albedo_times_color) {  // bmfr.cl:851-856 (for the PSNR references)
    return std::min(1.0, std::max(0.0, std::pow(std::max(0.0, (double)albedo_times_color), 0.454545)));
}

}  // namespace

// [start, end) of part i of n split into `parts` near-equal runs, multiples of
// 32 where possible (bmfr_amd/tiling.py _split: the same tiles as bench.py).
void split(int n, int parts, int i, int& a, int& b) {
    // std::nearbyint: ties to even, as Python's round()
    auto edge = [&](int k) { return k == parts ? n : (int)std::nearbyint((double)n * k / parts / 32.0) * 32; };
    a = edge(i);
    b = edge(i + 1);
}

// The frame loop over a tile grid: frame 0 per tile, then per frame the
// interior blocks of every tile, the halo exchange, the border blocks and
// TAA (bmfr_process_frame_interior / bmfr_exchange_run_all /
// bmfr_process_frame_border); each tile's output pixels are copied into the
// host frame.  Host frames are full-size; a tile uploads its region.
int run_tiled(const Options& o, const bmfr_config& base, const Camera& cam, const std::vector<std::vector<float>>& noisy,
              const std::vector<std::vector<float>>& normals, const std::vector<std::vector<float>>& positions,
              const std::vector<std::vector<float>>& albedos, std::vector<std::vector<float>>& out) {
    const int W = o.width, H = o.height, F = o.frames, T = o.tiles_x * o.tiles_y;
    if (o.gpus != 1 && o.gpus != T) {
        std::fprintf(stderr, "--gpus must be 1 or the number of tiles (%d)\n", T);
        return 1;
    }
    std::vector<int> tiles(4 * T);
    for (int r = 0; r < T; ++r) {
        int x0, x1, y0, y1;
        split(W, o.tiles_x, r % o.tiles_x, x0, x1);
        split(H, o.tiles_y, r / o.tiles_x, y0, y1);
        tiles[4 * r] = x0, tiles[4 * r + 1] = y0, tiles[4 * r + 2] = x1 - x0, tiles[4 * r + 3] = y1 - y0;
    }
    struct Tile {
        bmfr_config cfg;
        bmfr_ctx* ctx = nullptr;
        bmfr_sizes sz;
        int device = 0;
        hipStream_t stream = nullptr;
        hipEvent_t joined = nullptr;  // one-GPU runs: the stream join around the exchange
        float* in[2][4] = {};  // current / previous region planes: noisy, normal, position, albedo
        bmfr_exchange* x = nullptr;
    };
    std::vector<Tile> t(T);
    std::vector<bmfr_comm*> comms(T, nullptr);
    if (o.gpus == T && T > 1) {
        std::vector<int> devs(T);
        for (int r = 0; r < T; ++r) devs[r] = o.device + r;
        BMFR_CHECK(bmfr_comm_create_all(T, devs.data(), comms.data()));
    }
    for (int r = 0; r < T; ++r) {
        Tile& q = t[r];
        q.cfg = base;
        q.cfg.tile_x = tiles[4 * r], q.cfg.tile_y = tiles[4 * r + 1];
        q.cfg.tile_width = tiles[4 * r + 2], q.cfg.tile_height = tiles[4 * r + 3];
        q.cfg.tile_halo = o.tile_halo;
        q.device = o.gpus == T ? o.device + r : o.device;
        BMFR_CHECK(bmfr_create(&q.cfg, q.device, &q.ctx));
        BMFR_CHECK(bmfr_get_sizes(q.ctx, &q.sz));
        HIP_CHECK(hipSetDevice(q.device));
        HIP_CHECK(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&q.joined, hipEventDisableTiming));  // reused every frame
        for (auto& s : q.in)
            for (auto& p : s) HIP_CHECK(hipMalloc(&p, q.sz.region_bytes));
        BMFR_CHECK(bmfr_exchange_create(q.ctx, &q.cfg, tiles.data(), T, r, comms[r], &q.x));
    }
    std::printf("Processing %d frames (%dx%d) as %dx%d tiles, halo %d px, on %d GPU(s).\n", F, W, H, o.tiles_x,
                o.tiles_y, o.tile_halo, o.gpus);
    std::vector<bmfr_exchange*> xs(T);
    std::vector<void*> streams(T);
    for (int r = 0; r < T; ++r) xs[r] = t[r].x, streams[r] = t[r].stream;
    size_t sent = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int f = 0; f < F; ++f) {
        const int matrix_index = f == 0 ? 0 : f - 1;  // bmfr.cpp:440
        std::vector<bmfr_frame_inputs> in(T);
        for (int r = 0; r < T; ++r) {
            Tile& q = t[r];
            HIP_CHECK(hipSetDevice(q.device));
            const bmfr_sizes& z = q.sz;
            float** d = q.in[f & 1];
            const std::vector<float>* src[4] = {&noisy[f], &normals[f], &positions[f], &albedos[f]};
            for (int k = 0; k < 4; ++k)
                HIP_CHECK(hipMemcpy2DAsync(d[k], (size_t)z.region_width * 12,
                                           src[k]->data() + ((size_t)z.region_y * W + z.region_x) * 3, (size_t)W * 12,
                                           (size_t)z.region_width * 12, z.region_height, hipMemcpyHostToDevice,
                                           q.stream));
            float** pv = q.in[(f + 1) & 1];
            in[r] = {d[0], d[1], d[2], d[3], f > 0 ? pv[1] : nullptr, f > 0 ? pv[2] : nullptr};
        }
        if (f == 0) {
            for (int r = 0; r < T; ++r)
                BMFR_CHECK(bmfr_process_frame(t[r].ctx, t[r].stream, &in[r], &cam.matrices[16 * matrix_index],
                                              &cam.offsets[2 * f], f));
        } else {
            for (int r = 0; r < T; ++r)
                BMFR_CHECK(bmfr_process_frame_interior(t[r].ctx, t[r].stream, &in[r],
                                                       &cam.matrices[16 * matrix_index], &cam.offsets[2 * f], f));
            if (o.gpus == 1)  // one stream carries the device copies: join every tile's stream onto it
                for (int r = 1; r < T; ++r) {
                    HIP_CHECK(hipEventRecord(t[r].joined, t[r].stream));
                    HIP_CHECK(hipStreamWaitEvent(t[0].stream, t[r].joined, 0));
                }
            BMFR_CHECK(bmfr_exchange_run_all(xs.data(), T, streams.data(), f));
            if (o.gpus == 1) {
                HIP_CHECK(hipEventRecord(t[0].joined, t[0].stream));
                for (int r = 1; r < T; ++r) HIP_CHECK(hipStreamWaitEvent(t[r].stream, t[0].joined, 0));
            }
            for (int r = 0; r < T; ++r)
                BMFR_CHECK(bmfr_process_frame_border(t[r].ctx, t[r].stream, &in[r],
                                                     &cam.matrices[16 * matrix_index], &cam.offsets[2 * f], f));
            size_t s = 0;
            for (int r = 0; r < T; ++r) {
                size_t a = 0;
                (void)bmfr_exchange_bytes(t[r].x, f, &a, nullptr);
                s += a;
            }
            sent += s;
        }
        for (int r = 0; r < T; ++r) {  // the tile's pixels of the output (region row stride)
            Tile& q = t[r];
            const bmfr_sizes& z = q.sz;
            const float* res = bmfr_output(q.ctx);
            const int tx = tiles[4 * r], ty = tiles[4 * r + 1], tw = tiles[4 * r + 2], th = tiles[4 * r + 3];
            HIP_CHECK(hipSetDevice(q.device));
            HIP_CHECK(hipMemcpy2DAsync(out[f].data() + ((size_t)ty * W + tx) * 3, (size_t)W * 12,
                                       res + ((size_t)(ty - z.region_y) * z.region_width + (tx - z.region_x)) * 3,
                                       (size_t)z.region_width * 12, (size_t)tw * 12, th, hipMemcpyDeviceToHost,
                                       q.stream));
            // the region buffers of frame f are read again as frame f+1's previous planes
            // and rewritten by frame f+2: finish the frame before its slot is reused
        }
        for (int r = 0; r < T; ++r) {
            HIP_CHECK(hipSetDevice(t[r].device));
            HIP_CHECK(hipStreamSynchronize(t[r].stream));
        }
    }
    const double wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    int rc = 0;
    for (int r = 0; r < T; ++r) {
        unsigned over = 0;
        const bmfr_status st = bmfr_halo_status(t[r].ctx, &over);
        if (st != BMFR_OK) {
            std::printf("tile %d: %s (%u px)\n", r, bmfr_status_string(st), over);
            rc = 1;
        }
    }
    std::printf("Tiled: %.3f ms/frame wall (synchronous per frame), halo %.2f MB sent per frame\n", wall_ms / F,
                F > 1 ? sent / 1e6 / (F - 1) : 0.0);
    for (int r = 0; r < T; ++r) {
        Tile& q = t[r];
        HIP_CHECK(hipSetDevice(q.device));
        bmfr_exchange_destroy(q.x);
        for (auto& s : q.in)
            for (auto& p : s) (void)hipFree(p);
        (void)hipStreamDestroy(q.stream);
        (void)hipEventDestroy(q.joined);
        bmfr_destroy(q.ctx);
        if (comms[r]) bmfr_comm_destroy(comms[r]);
    }
    return rc;
}

int run(const Options& o) {
    const int W = o.width, H = o.height, F = o.frames;
    const size_t plane = (size_t)W * H * 3;
    Camera cam;
    cam.matrices.resize((size_t)F * 16);
    cam.offsets.resize((size_t)F * 2);

    if (!o.write_synthetic.empty()) {
        std::printf("Writing a %dx%d, %d-frame synthetic dataset to %s\n", W, H, F, o.write_synthetic.c_str());
        bool ok = true;
#pragma omp parallel for
        for (int f = 0; f < F; ++f) {
            std::vector<float> n(plane), nr(plane), p(plane), a(plane);
            if (bmfr_synth_frame_host(W, H, f, o.seed, n.data(), nr.data(), p.data(), a.data(), nullptr) != BMFR_OK) {
                ok = false;
                continue;
            }
            const std::string d = o.write_synthetic;
            const struct {
                const char* name;
                const float* data;
            } files[] = {{NOISY_FILE_NAME, n.data()}, {NORMAL_FILE_NAME, nr.data()},
                         {POSITION_FILE_NAME, p.data()}, {ALBEDO_FILE_NAME, a.data()}};
            for (const auto& fl : files)
                if (bmfr_exr_write_rgb(frame_file(d + fl.name, f, ".exr").c_str(), W, H, fl.data, (size_t)W * 3,
                                       BMFR_EXR_ZIP) != 0)
                    ok = false;
        }
        for (int f = 0; f < F; ++f) {
            float m[16], off[2];
            bmfr_synth_camera(W, H, f, m, off);
            std::copy(m, m + 16, cam.matrices.begin() + 16 * f);
            std::copy(off, off + 2, cam.offsets.begin() + 2 * f);
        }
        // The synthetic scene's limits (bmfr_config_default).
        if (!ok || !write_camera(o.write_synthetic + "/camera_matrices.h", F, cam)) {
            std::fprintf(stderr, "writing the dataset failed: %s\n", bmfr_io_error());
            return 1;
        }
        return 0;
    }

    std::printf("Initialize.\n");
    bmfr_config cfg;
    bmfr_config_default(&cfg, W, H);
    std::vector<int> ns, sc;
    if (!parse_features(o.not_scaled, ns) || !parse_features(o.scaled, sc)) return 1;
    cfg.features_not_scaled = (int)ns.size();
    cfg.features_scaled = (int)sc.size();
    for (size_t i = 0; i < ns.size() + sc.size() && i < BMFR_MAX_FEATURES; ++i)
        cfg.feature_buffers[i] = i < ns.size() ? ns[i] : sc[i - ns.size()];
    cfg.noise_amount = NOISE_AMOUNT;
    cfg.blend_alpha = BLEND_ALPHA;
    cfg.second_blend_alpha = SECOND_BLEND_ALPHA;
    cfg.taa_blend_alpha = TAA_BLEND_ALPHA;
    cfg.use_half_precision_in_tmp_data = o.half_tmp;

    if (o.synthetic) {
        for (int f = 0; f < F; ++f) bmfr_synth_camera(W, H, f, &cam.matrices[16 * f], &cam.offsets[2 * f]);
    } else if (!load_camera(o.camera, F, cam)) {
        std::fprintf(stderr, "cannot read %d frames of camera data from %s\n", F, o.camera.c_str());
        return 1;
    } else {
        cfg.position_limit_squared = cam.position_limit_squared;
        cfg.normal_limit_squared = cam.normal_limit_squared;
    }

    cfg.fast_fit = o.fast_fit;
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, o.device));
    std::printf("Using device named: %s\n", prop.name);
    const bool tiled = o.tiles_x > 0;
    bmfr_ctx* ctx = nullptr;
    if (!tiled) BMFR_CHECK(bmfr_create(&cfg, o.device, &ctx));

    // ---- Loading input data (bmfr.cpp:254-307) ----
    std::printf("Loading input data.\n");
    std::vector<std::vector<float>> albedos(F), normals(F), positions(F), noisy(F), out(F);
    bool error = false;
#pragma omp parallel for
    for (int f = 0; f < F; ++f) {
        if (error) continue;
        albedos[f].resize(plane);
        normals[f].resize(plane);
        positions[f].resize(plane);
        noisy[f].resize(plane);
        out[f].resize(plane);
        if (o.synthetic) {
            if (bmfr_synth_frame_host(W, H, f, o.seed, noisy[f].data(), normals[f].data(), positions[f].data(),
                                      albedos[f].data(), nullptr) != BMFR_OK)
                error = true;
            continue;
        }
        const struct {
            const char* name;
            std::vector<float>* v;
        } files[] = {{ALBEDO_FILE_NAME, &albedos[f]}, {NORMAL_FILE_NAME, &normals[f]},
                     {POSITION_FILE_NAME, &positions[f]}, {NOISY_FILE_NAME, &noisy[f]}};
        for (const auto& fl : files) {
            if (bmfr_exr_read_rgb(frame_file(o.input + fl.name, f, ".exr").c_str(), W, H, fl.v->data()) != 0) {
#pragma omp critical
                std::printf("Buffer loading failed, reason: %s\n", bmfr_io_error());
                error = true;
                break;
            }
        }
    }
    if (error) {
        std::printf("One or more errors occurred during buffer loading\n");
        if (ctx) bmfr_destroy(ctx);
        return 1;
    }
    if (tiled) {
        const int rc = run_tiled(o, cfg, cam, noisy, normals, positions, albedos, out);
        if (rc != 0) return rc;
        bool err = false;
        if (o.save) {
#pragma omp parallel for
            for (int f = 0; f < F; ++f) {
                const std::string name = frame_file(o.output, f, o.exr ? ".exr" : ".png");
                const int r = o.exr ? bmfr_exr_write_rgb(name.c_str(), W, H, out[f].data(), (size_t)W * 3, BMFR_EXR_ZIP)
                                    : bmfr_png_write_rgb(name.c_str(), W, H, out[f].data(), (size_t)W * 3);
                if (r != 0) err = true;
            }
        }
        return err ? 1 : 0;
    }

    // ---- Device buffers: a ring of 3 input sets (frame f, f-1 as the
    // previous normals/positions, f+1 uploading) ----
    constexpr int kRing = 3;
    float* dev[kRing][4];
    for (auto& s : dev)
        for (auto& p : s) HIP_CHECK(hipMalloc(&p, plane * sizeof(float)));
    hipStream_t compute, copy;
    HIP_CHECK(hipStreamCreateWithFlags(&compute, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&copy, hipStreamNonBlocking));
    std::vector<hipEvent_t> uploaded(F), consumed(F);
    for (int f = 0; f < F; ++f) {
        HIP_CHECK(hipEventCreateWithFlags(&uploaded[f], hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&consumed[f], hipEventDisableTiming));
    }
    // Page-lock the host frames so uploads and readbacks are asynchronous DMA.
    std::vector<void*> registered;
    if (o.pipelined) {
        for (auto* vs : {&albedos, &normals, &positions, &noisy, &out})
            for (auto& v : *vs)
                if (hipHostRegister(v.data(), plane * sizeof(float), hipHostRegisterDefault) == hipSuccess)
                    registered.push_back(v.data());
    }
    auto upload = [&](int f) -> hipError_t {
        hipStream_t s = o.pipelined ? copy : compute;
        // Slot f % 3 was last read by frame f-3 (as current) and frame f-2 (as
        // previous); upload(f) is issued after frame f-2 was enqueued, so
        // consumed[f-2] is recorded (an unrecorded event would not be waited on).
        if (f >= 2) {
            hipError_t e = hipStreamWaitEvent(s, consumed[f - 2], 0);
            if (e != hipSuccess) return e;
        }
        float** d = dev[f % kRing];
        const std::vector<float>* src[4] = {&noisy[f], &normals[f], &positions[f], &albedos[f]};
        for (int k = 0; k < 4; ++k) {
            hipError_t e = hipMemcpyAsync(d[k], src[k]->data(), plane * sizeof(float), hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return e;
        }
        return hipEventRecord(uploaded[f], s);
    };

    BMFR_CHECK(bmfr_set_profiling(ctx, 1, F));
    std::printf("Processing %d frames (%dx%d, B=%d).\n", F, W, H, cfg.features_not_scaled + cfg.features_scaled + 3);
    const auto t0 = std::chrono::steady_clock::now();
    HIP_CHECK(upload(0));
    for (int f = 0; f < F; ++f) {
        if (f + 1 < F) HIP_CHECK(upload(f + 1));  // overlaps frame f
        HIP_CHECK(hipStreamWaitEvent(compute, uploaded[f], 0));
        float** d = dev[f % kRing];
        float** pv = dev[(f + kRing - 1) % kRing];
        bmfr_frame_inputs in = {d[0], d[1], d[2], d[3], f > 0 ? pv[1] : nullptr, f > 0 ? pv[2] : nullptr};
        const int matrix_index = f == 0 ? 0 : f - 1;  // bmfr.cpp:440
        BMFR_CHECK(bmfr_process_frame(ctx, compute, &in, &cam.matrices[16 * matrix_index], &cam.offsets[2 * f], f));
        HIP_CHECK(hipEventRecord(consumed[f], compute));
        // Not timed upstream either: the result goes to the frame buffer (bmfr.cpp:478-480).
        HIP_CHECK(hipMemcpyAsync(out[f].data(), bmfr_output(ctx), plane * sizeof(float), hipMemcpyDeviceToHost,
                                 compute));
    }
    HIP_CHECK(hipStreamSynchronize(compute));
    const double wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    // ---- Profiling report (bmfr.cpp:488-517: frame 0 excluded from the temporal stages) ----
    std::vector<bmfr_frame_profile> prof(F);
    int n = 0;
    BMFR_CHECK(bmfr_get_profile(ctx, prof.data(), F, &n));
    double k1 = 0, k2 = 0, tot = 0;
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (prof[i].frame_number > 0) {
            k1 += prof[i].fused_block_ms;
            k2 += prof[i].taa_ms;
            tot += prof[i].total_ms;
            ++m;
        }
    if (m > 0) {
        std::printf("fused accumulate+fitter+weighted_sum+accumulate_filtered (K1): mean %.4f ms\n", k1 / m);
        std::printf("taa (K2): mean %.4f ms\n", k2 / m);
        std::printf("Total (device, frames 1..%d): mean %.4f ms\n", F - 1, tot / m);
    }
    std::printf("Wall time incl. uploads and readbacks: %.2f ms for %d frames (%.3f ms/frame, %s)\n", wall_ms, F,
                wall_ms / F, o.pipelined ? "pipelined" : "synchronous");

    // ---- PSNR against reference images ----
    if (!o.psnr.empty()) {
        double sum = 0;
        int cnt = 0;
        std::vector<float> ref(plane);
        for (int f = 0; f < F; ++f) {
            if (bmfr_exr_read_rgb(frame_file(o.psnr, f, ".exr").c_str(), W, H, ref.data()) != 0) {
                std::printf("PSNR: %s\n", bmfr_io_error());
                break;
            }
            double mse = 0;
            for (size_t i = 0; i < plane; ++i) {
                const double d = (double)out[f][i] - tonemap(ref[i]);
                mse += d * d;
            }
            mse /= (double)plane;
            const double p = mse > 0 ? 10.0 * std::log10(1.0 / mse) : 99.0;
            sum += p;
            ++cnt;
        }
        if (cnt) std::printf("PSNR vs %s*: mean %.3f dB over %d frames\n", o.psnr.c_str(), sum / cnt, cnt);
    }

    // ---- Store results (bmfr.cpp:519-553) ----
    if (o.save) {
        error = false;
#pragma omp parallel for
        for (int f = 0; f < F; ++f) {
            const std::string name = frame_file(o.output, f, o.exr ? ".exr" : ".png");
            const int r = o.exr ? bmfr_exr_write_rgb(name.c_str(), W, H, out[f].data(), (size_t)W * 3, BMFR_EXR_ZIP)
                                : bmfr_png_write_rgb(name.c_str(), W, H, out[f].data(), (size_t)W * 3);
            if (r != 0) {
#pragma omp critical
                std::printf("Can't create image file on disk to location %s\n", name.c_str());
                error = true;
            }
        }
        if (error) std::printf("One or more errors occurred during image saving\n");
    }

    for (void* p : registered) (void)hipHostUnregister(p);
    for (auto& s : dev)
        for (auto& p : s) (void)hipFree(p);
    for (int f = 0; f < F; ++f) {
        (void)hipEventDestroy(uploaded[f]);
        (void)hipEventDestroy(consumed[f]);
    }
    (void)hipStreamDestroy(compute);
    (void)hipStreamDestroy(copy);
    bmfr_destroy(ctx);
    return error ? 1 : 0;
}

int main(int argc, char** argv) {
    Options o;
    if (!parse_args(argc, argv, o)) return 2;
    return run(o);
}
