// bmfr_synth.hip -- deterministic synthetic 1-spp frames (stands in for the
// external 60-frame EXR dataset of bmfr.cpp:42-53, which is not available).
//
// Scene: a closed room (|x|,|z| <= 14, -2 <= y <= 12) with eight spheres, so
// every ray hits and |world_position| <= 16 per axis (p^3 stays finite in
// half, cf. bmfr.cpp:85-87).  Outputs per pixel: shading normal, world
// position, albedo (procedural checker in [0.1, 0.9]), demodulated noisy
// irradiance = clean irradiance x Exp(1) per channel with rare x50 fireflies,
// and optionally the clean tone-mapped image (the PSNR reference).
// Camera: slow dolly + yaw; camera_matrices[f] is the column-major
// view-projection of frame f, pixel_offsets[f] a Halton(2,3) jitter.  The
// primary ray of pixel (x,y) goes through NDC (2(x+jx)/W-1, 2(y+1-jy)/H-1),
// the inverse of the reprojection of bmfr.cl:343-355.
#include <cmath>
#include <cstring>

#include <hip/hip_runtime.h>

#include "../../include/bmfr.h"

#define HD __host__ __device__

namespace {

struct V3 {
    float x, y, z;
};
HD inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
HD inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
HD inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
HD inline V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
HD inline float dotv(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct CameraBasis {
    V3 eye, right, up, fwd;
    float tan_x, tan_y;
    float jx, jy;
};

constexpr int kSpheres = 8;
struct Sphere {
    float cx, cy, cz, r, ar, ag, ab;
};
__host__ __device__ inline Sphere sphere(int i) {
    // centre, radius, albedo
    const Sphere s[kSpheres] = {
        {-4.f, 0.f, -2.f, 2.f, 0.80f, 0.25f, 0.20f},  {3.f, -0.5f, -4.f, 1.5f, 0.20f, 0.70f, 0.30f},
        {0.f, 1.5f, -8.f, 3.5f, 0.75f, 0.75f, 0.70f}, {6.f, 0.5f, 2.f, 2.5f, 0.25f, 0.35f, 0.85f},
        {-7.f, 1.f, -7.f, 3.f, 0.85f, 0.80f, 0.20f},  {1.5f, -1.f, 1.f, 1.f, 0.60f, 0.30f, 0.80f},
        {-2.f, 4.f, -5.f, 1.2f, 0.30f, 0.80f, 0.80f}, {8.f, 3.f, -8.f, 2.2f, 0.90f, 0.55f, 0.30f}};
    return s[i];
}

constexpr float kRoomX = 14.f, kRoomZ = 14.f, kFloor = -2.f, kCeil = 12.f;

HD inline double halton(int index, int base) {
    double f = 1.0, r = 0.0;
    while (index > 0) {
        f /= base;
        r += f * (index % base);
        index /= base;
    }
    return r;
}

HD inline uint32_t mix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

// Camera of frame f in double precision (host), like a renderer would export it.
void camera_frame(int W, int H, int f, double eye[3], double right[3], double up[3], double fwd[3],
                  double* tan_x, double* tan_y) {
    // Slow pan + dolly: about 1.1 px/frame at 960 px wide (4.5 at 3840),
    // proportional to the resolution like a real camera (SURVEY.md 8d asks
    // for a slow pan; the tiled path's halo must cover this motion).
    const double yaw = 0.35 - 0.0003 * f, pitch = -0.12 + 0.0001 * f;
    eye[0] = -2.0 + 0.003 * f;
    eye[1] = 2.0 + 0.0005 * f;
    eye[2] = 9.0 - 0.00625 * f;
    fwd[0] = -std::sin(yaw) * std::cos(pitch);
    fwd[1] = std::sin(pitch);
    fwd[2] = -std::cos(yaw) * std::cos(pitch);
    // right = normalize(cross(fwd, world_up)), up = cross(right, fwd)
    right[0] = -fwd[2];
    right[1] = 0.0;
    right[2] = fwd[0];
    const double rl = std::sqrt(right[0] * right[0] + right[2] * right[2]);
    right[0] /= rl;
    right[2] /= rl;
    up[0] = right[1] * fwd[2] - right[2] * fwd[1];
    up[1] = right[2] * fwd[0] - right[0] * fwd[2];
    up[2] = right[0] * fwd[1] - right[1] * fwd[0];
    const double fovy = 50.0 * 3.14159265358979323846 / 180.0;
    *tan_y = std::tan(fovy / 2);
    *tan_x = *tan_y * (double)W / (double)H;
}

CameraBasis basis(int W, int H, int f) {
    double e[3], r[3], u[3], fw[3], tx, ty;
    camera_frame(W, H, f, e, r, u, fw, &tx, &ty);
    CameraBasis b;
    b.eye = v3((float)e[0], (float)e[1], (float)e[2]);
    b.right = v3((float)r[0], (float)r[1], (float)r[2]);
    b.up = v3((float)u[0], (float)u[1], (float)u[2]);
    b.fwd = v3((float)fw[0], (float)fw[1], (float)fw[2]);
    b.tan_x = (float)tx;
    b.tan_y = (float)ty;
    b.jx = (float)halton(f + 1, 2);
    b.jy = (float)halton(f + 1, 3);
    return b;
}

struct Hit {
    V3 p, n, albedo;
};

HD inline Hit trace(V3 o, V3 d) {
    float best = 1e30f;
    int which = -1;
    for (int i = 0; i < kSpheres; ++i) {
        const Sphere s = sphere(i);
        const V3 oc = sub(o, v3(s.cx, s.cy, s.cz));
        const float b = dotv(oc, d);
        const float c = dotv(oc, oc) - s.r * s.r;
        const float disc = b * b - c;
        if (disc > 0.f) {
            const float t = -b - sqrtf(disc);
            if (t > 1e-3f && t < best) {
                best = t;
                which = i;
            }
        }
    }
    // walls (camera is inside the box, so exactly one exit per axis)
    int wall = -1;
    const float tx = ((d.x > 0.f ? kRoomX : -kRoomX) - o.x) / d.x;
    const float ty = ((d.y > 0.f ? kCeil : kFloor) - o.y) / d.y;
    const float tz = ((d.z > 0.f ? kRoomZ : -kRoomZ) - o.z) / d.z;
    if (tx > 0.f && tx < best) { best = tx; wall = 0; which = -1; }
    if (ty > 0.f && ty < best) { best = ty; wall = 1; which = -1; }
    if (tz > 0.f && tz < best) { best = tz; wall = 2; which = -1; }
    Hit h;
    h.p = add(o, mul(d, best));
    if (which >= 0) {
        const Sphere s = sphere(which);
        h.n = mul(sub(h.p, v3(s.cx, s.cy, s.cz)), 1.f / s.r);
        h.albedo = v3(s.ar, s.ag, s.ab);
    } else {
        // inward-facing wall normal, checker albedo in [0.1, 0.9]
        h.n = v3(wall == 0 ? (d.x > 0.f ? -1.f : 1.f) : 0.f, wall == 1 ? (d.y > 0.f ? -1.f : 1.f) : 0.f,
                 wall == 2 ? (d.z > 0.f ? -1.f : 1.f) : 0.f);
        const int chk = ((int)floorf(h.p.x * 0.5f) + (int)floorf(h.p.y * 0.5f) + (int)floorf(h.p.z * 0.5f)) & 1;
        const float a = chk ? 0.85f : 0.15f;
        const V3 tint = wall == 1 ? v3(1.f, 0.92f, 0.8f) : (wall == 0 ? v3(0.9f, 1.f, 0.95f) : v3(0.95f, 0.95f, 1.f));
        h.albedo = v3(0.1f + (a - 0.1f) * tint.x, 0.1f + (a - 0.1f) * tint.y, 0.1f + (a - 0.1f) * tint.z);
    }
    return h;
}

HD inline V3 irradiance(V3 p, V3 n) {
    const V3 lp[2] = {v3(0.f, 10.f, 0.f), v3(-10.f, 6.f, 8.f)};
    const V3 li[2] = {v3(60.f, 57.f, 51.f), v3(18.f, 21.f, 30.f)};
    V3 e = v3(0.08f, 0.08f, 0.09f);
    for (int k = 0; k < 2; ++k) {
        const V3 l = sub(lp[k], p);
        const float d2 = dotv(l, l);
        const float cosv = dotv(n, l) / sqrtf(d2);
        if (cosv > 0.f) e = add(e, mul(li[k], cosv / (1.f + d2)));
    }
    return e;
}

// Pixel (x, y) of the W x H frame, stored at element 3*o of the planes.
HD inline void shade_pixel(int W, int H, int x, int y, long o, int frame, uint32_t seed, const CameraBasis& b,
                           float* noisy, float* normals, float* positions, float* albedo, float* clean) {
    const float nx = 2.f * ((float)x + b.jx) / (float)W - 1.f;
    const float ny = 2.f * ((float)y + 1.f - b.jy) / (float)H - 1.f;
    V3 d = add(add(b.fwd, mul(b.right, nx * b.tan_x)), mul(b.up, ny * b.tan_y));
    d = mul(d, 1.f / sqrtf(dotv(d, d)));
    const Hit h = trace(b.eye, d);
    const V3 e = irradiance(h.p, h.n);
    const long i = 3L * o;
    float ec[3] = {e.x, e.y, e.z};
    const uint32_t base = mix32(seed ^ mix32((uint32_t)frame * 0x9E3779B1u + 0x632BE5ABu)) ^
                          (uint32_t)((long)y * W + x) * 0x85EBCA77u;
    const uint32_t fire = mix32(base ^ 0x27d4eb2fu);
    const float firefly = fire < 429497u ? 50.f : 1.f;  // p = 1e-4
    for (int c = 0; c < 3; ++c) {
        const uint32_t r = mix32(base + 0xC2B2AE3Du * (uint32_t)(c + 1));
        const float u = ((float)(r >> 8) + 1.f) * (1.f / 16777216.f);  // (0, 1]
        noisy[i + c] = ec[c] * (-logf(u)) * firefly;
    }
    normals[i] = h.n.x;
    normals[i + 1] = h.n.y;
    normals[i + 2] = h.n.z;
    positions[i] = h.p.x;
    positions[i + 1] = h.p.y;
    positions[i + 2] = h.p.z;
    albedo[i] = h.albedo.x;
    albedo[i + 1] = h.albedo.y;
    albedo[i + 2] = h.albedo.z;
    if (clean) {
        const float a[3] = {h.albedo.x, h.albedo.y, h.albedo.z};
        for (int c = 0; c < 3; ++c) {
            const float v = powf(fmaxf(0.f, a[c] * ec[c]), 0.454545f);
            clean[i + c] = fminf(fmaxf(v, 0.f), 1.f);
        }
    }
}

// The region [x0, x0 + rw) x [y0, y0 + rh) of the frame, planes of row stride rw.
__global__ void k_synth(int W, int H, int x0, int y0, int rw, int rh, int frame, uint32_t seed, CameraBasis b,
                        float* noisy, float* normals, float* positions, float* albedo, float* clean) {
    const int rx = blockIdx.x * blockDim.x + threadIdx.x;
    const int ry = blockIdx.y * blockDim.y + threadIdx.y;
    if (rx >= rw || ry >= rh) return;
    shade_pixel(W, H, x0 + rx, y0 + ry, (long)ry * rw + rx, frame, seed, b, noisy, normals, positions, albedo,
                clean);
}

}  // namespace

extern "C" {

void bmfr_synth_camera(int W, int H, int f, float vp[16], float off[2]) {
    double e[3], r[3], u[3], fw[3], tx, ty;
    camera_frame(W, H, f, e, r, u, fw, &tx, &ty);
    // View: rows right, up, -fwd; projection: GL perspective with these
    // tangents.  VP = P * V, stored column-major (m[col*4 + row]).
    const double n = 0.05, fa = 100.0;
    double V[4][4] = {{r[0], r[1], r[2], -(r[0] * e[0] + r[1] * e[1] + r[2] * e[2])},
                      {u[0], u[1], u[2], -(u[0] * e[0] + u[1] * e[1] + u[2] * e[2])},
                      {-fw[0], -fw[1], -fw[2], (fw[0] * e[0] + fw[1] * e[1] + fw[2] * e[2])},
                      {0, 0, 0, 1}};
    double P[4][4] = {{1.0 / tx, 0, 0, 0},
                      {0, 1.0 / ty, 0, 0},
                      {0, 0, (fa + n) / (n - fa), 2 * fa * n / (n - fa)},
                      {0, 0, -1, 0}};
    for (int row = 0; row < 4; ++row)
        for (int col = 0; col < 4; ++col) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += P[row][k] * V[k][col];
            vp[col * 4 + row] = (float)s;
        }
    off[0] = (float)halton(f + 1, 2);
    off[1] = (float)halton(f + 1, 3);
}

bmfr_status bmfr_synth_frame_host(int W, int H, int frame, uint32_t seed, float* noisy, float* normals,
                                  float* positions, float* albedo, float* clean) {
    if (W <= 0 || H <= 0 || frame < 0 || !noisy || !normals || !positions || !albedo)
        return BMFR_ERROR_INVALID_ARGUMENT;
    const CameraBasis b = basis(W, H, frame);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            shade_pixel(W, H, x, y, (long)y * W + x, frame, seed, b, noisy, normals, positions, albedo, clean);
    return BMFR_OK;
}

bmfr_status bmfr_synth_region_device(int W, int H, int x0, int y0, int rw, int rh, int frame, uint32_t seed,
                                     float* noisy, float* normals, float* positions, float* albedo, float* clean,
                                     void* stream) {
    if (W <= 0 || H <= 0 || frame < 0 || !noisy || !normals || !positions || !albedo || x0 < 0 || y0 < 0 ||
        rw <= 0 || rh <= 0 || x0 + rw > W || y0 + rh > H)
        return BMFR_ERROR_INVALID_ARGUMENT;
    const CameraBasis b = basis(W, H, frame);
    const dim3 blk(64, 4), grd((rw + 63) / 64, (rh + 3) / 4);
    hipLaunchKernelGGL(k_synth, grd, blk, 0, reinterpret_cast<hipStream_t>(stream), W, H, x0, y0, rw, rh, frame,
                       seed, b, noisy, normals, positions, albedo, clean);
    return hipGetLastError() == hipSuccess ? BMFR_OK : BMFR_ERROR_HIP;
}

bmfr_status bmfr_synth_frame_device(int W, int H, int frame, uint32_t seed, float* noisy, float* normals,
                                    float* positions, float* albedo, float* clean, void* stream) {
    return bmfr_synth_region_device(W, H, 0, 0, W, H, frame, seed, noisy, normals, positions, albedo, clean,
                                    stream);
}

}  // extern "C"
