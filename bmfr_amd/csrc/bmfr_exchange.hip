// bmfr_exchange.hip -- the multi-GPU halo exchange behind the C ABI
// (include/bmfr.h, "Multi-GPU halo exchange"): the per-frame plan of a tile
// grid (bmfr_halo_plan), RCCL communicators (bmfr_comm_*) and the exchange
// itself (bmfr_exchange_*): one pack kernel, one grouped ncclSend / ncclRecv
// batch to the neighbouring tiles over xGMI, one unpack kernel, all on the
// caller's stream -- one C call per frame, no host work on the frame path
// beyond enqueueing.  No reference counterpart: the reference runs one GPU
// ("Distributed communication backend").
//
// RCCL is loaded at run time (dlopen): the process's own copy if one is
// already mapped (torch's), else /opt/rocm's librccl.so.1, so libbmfr itself
// carries no link dependency on it.
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/bmfr.h"

namespace {

// ---------------------------------------------------------------- RCCL ----
struct NcclId {
    char internal[128];  // ncclUniqueId (rccl.h: NCCL_UNIQUE_ID_BYTES)
};
constexpr int kNcclUint8 = 1;  // ncclDataType_t ncclUint8

struct Rccl {
    void* handle = nullptr;
    int (*get_unique_id)(NcclId*) = nullptr;
    int (*comm_init_rank)(void**, int, NcclId, int) = nullptr;
    int (*comm_init_all)(void**, int, const int*) = nullptr;
    int (*comm_destroy)(void*) = nullptr;
    int (*group_start)() = nullptr;
    int (*group_end)() = nullptr;
    int (*send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
    int (*recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
    bool ok = false;
};

Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        for (const char* name : {"librccl.so.1", "librccl.so"}) {  // a copy already mapped (torch's)
            if ((x.handle = dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
        }
        if (!x.handle) x.handle = dlopen("librccl.so.1", RTLD_NOW);
        if (!x.handle) x.handle = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!x.handle) return x;
        auto sym = [&](auto& f, const char* n) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(x.handle, n)); };
        sym(x.get_unique_id, "ncclGetUniqueId");
        sym(x.comm_init_rank, "ncclCommInitRank");
        sym(x.comm_init_all, "ncclCommInitAll");
        sym(x.comm_destroy, "ncclCommDestroy");
        sym(x.group_start, "ncclGroupStart");
        sym(x.group_end, "ncclGroupEnd");
        sym(x.send, "ncclSend");
        sym(x.recv, "ncclRecv");
        x.ok = x.get_unique_id && x.comm_init_rank && x.comm_init_all && x.comm_destroy && x.group_start &&
               x.group_end && x.send && x.recv;
        return x;
    }();
    return r;
}

bmfr_status hip_st(hipError_t e) { return e == hipSuccess ? BMFR_OK : BMFR_ERROR_HIP; }

// ---------------------------------------------------------------- plan ----
struct Rect {
    int x, y, w, h;
    bool empty() const { return w <= 0 || h <= 0; }
};

Rect intersect(Rect a, Rect b) {
    const int x0 = std::max(a.x, b.x), y0 = std::max(a.y, b.y);
    const int x1 = std::min(a.x + a.w, b.x + b.w), y1 = std::min(a.y + a.h, b.y + b.h);
    return Rect{x0, y0, x1 - x0, y1 - y0};
}

// The bmfr_halo_copy records for the part of `part` a frame reads: inside the
// state rectangle (three accumulation planes) and / or the result rectangle
// (TAA output); one record with every plane when both parts coincide.
void masked(Rect part, Rect state, Rect result, std::vector<int>& out) {
    const Rect s = intersect(part, state), r = intersect(part, result);
    auto put = [&](Rect q, int planes) { out.insert(out.end(), {q.x, q.y, q.w, q.h, planes}); };
    if (!s.empty() && !r.empty() && s.x == r.x && s.y == r.y && s.w == r.w && s.h == r.h) {
        put(s, BMFR_HALO_ALL);
        return;
    }
    if (!s.empty()) put(s, BMFR_HALO_STATE);
    if (!r.empty()) put(r, BMFR_HALO_RESULT);
}

bmfr_status need_of(const bmfr_config* cfg, const int* t, int frame, Rect& st, Rect& rs) {
    bmfr_config c = *cfg;
    c.tile_x = t[0], c.tile_y = t[1], c.tile_width = t[2], c.tile_height = t[3];
    int a[4], b[4];
    const bmfr_status s = bmfr_halo_need(&c, frame, a, b);
    st = Rect{a[0], a[1], a[2], a[3]};
    rs = Rect{b[0], b[1], b[2], b[3]};
    return s;
}

struct PeerPlan {
    int peer;
    std::vector<int> send, recv;  // bmfr_halo_copy records
    size_t send_bytes = 0, recv_bytes = 0;
};

// TileGrid.frame_plan (bmfr_amd/tiling.py): for every other tile, the parts
// of my tile its frame reads (send) and the parts of its tile mine reads (recv).
bmfr_status make_plan(const bmfr_config* cfg, const int* tiles, int ntiles, int rank, int frame,
                      std::vector<PeerPlan>& out) {
    out.clear();
    std::vector<Rect> st(ntiles), rs(ntiles);
    for (int r = 0; r < ntiles; ++r) {
        const bmfr_status s = need_of(cfg, tiles + 4 * r, frame, st[r], rs[r]);
        if (s != BMFR_OK) return s;
    }
    const Rect mine{tiles[4 * rank], tiles[4 * rank + 1], tiles[4 * rank + 2], tiles[4 * rank + 3]};
    for (int p = 0; p < ntiles; ++p) {
        if (p == rank) continue;
        PeerPlan pp;
        pp.peer = p;
        masked(mine, st[p], rs[p], pp.send);
        const Rect theirs{tiles[4 * p], tiles[4 * p + 1], tiles[4 * p + 2], tiles[4 * p + 3]};
        masked(theirs, st[rank], rs[rank], pp.recv);
        if (!pp.send.empty() || !pp.recv.empty()) out.push_back(std::move(pp));
    }
    return BMFR_OK;
}

bmfr_status validate_grid(const bmfr_config* cfg, const int* tiles, int ntiles, int rank) {
    if (!cfg || !tiles || ntiles < 1 || rank < 0 || rank >= ntiles) return BMFR_ERROR_INVALID_ARGUMENT;
    // the tiles must partition the frame (each pixel in exactly one tile)
    long long area = 0;
    for (int r = 0; r < ntiles; ++r) {
        const int* t = tiles + 4 * r;
        if (t[2] <= 0 || t[3] <= 0 || t[0] < 0 || t[1] < 0 || t[0] + t[2] > cfg->image_width ||
            t[1] + t[3] > cfg->image_height)
            return BMFR_ERROR_INVALID_ARGUMENT;
        area += (long long)t[2] * t[3];
        for (int q = 0; q < r; ++q) {
            const int* u = tiles + 4 * q;
            if (!intersect(Rect{t[0], t[1], t[2], t[3]}, Rect{u[0], u[1], u[2], u[3]}).empty())
                return BMFR_ERROR_INVALID_ARGUMENT;
        }
    }
    return area == (long long)cfg->image_width * cfg->image_height ? BMFR_OK : BMFR_ERROR_INVALID_ARGUMENT;
}

}  // namespace

struct bmfr_comm {
    void* nccl = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

struct bmfr_exchange {
    bmfr_ctx* ctx = nullptr;
    bmfr_comm* comm = nullptr;
    int rank = 0, ntiles = 0;
    std::vector<PeerPlan> plans[16];  // per frame % 16 (the block grid's shift)
    std::vector<int> send_all[16], recv_all[16];
    size_t send_total[16] = {}, recv_total[16] = {};
    uint8_t* sbuf = nullptr;
    uint8_t* rbuf = nullptr;
    size_t scap = 0, rcap = 0;
    int device = 0;
};

extern "C" {

bmfr_status bmfr_halo_plan(const bmfr_config* cfg, const int* tiles, int ntiles, int rank, int frame_number,
                           int* peers, int* send_counts, int* recv_counts, int* records, int max_records,
                           int* n_peers) {
    if (frame_number < 0 || !n_peers) return BMFR_ERROR_INVALID_ARGUMENT;
    bmfr_status s = validate_grid(cfg, tiles, ntiles, rank);
    if (s != BMFR_OK) return s;
    std::vector<PeerPlan> plan;
    if ((s = make_plan(cfg, tiles, ntiles, rank, frame_number, plan)) != BMFR_OK) return s;
    *n_peers = (int)plan.size();
    int nrec = 0;
    for (const auto& p : plan) nrec += (int)(p.send.size() + p.recv.size()) / 5;
    if (!peers && !records) return BMFR_OK;  // sizes only
    if (!peers || !send_counts || !recv_counts || !records || nrec > max_records) return BMFR_ERROR_INVALID_ARGUMENT;
    int k = 0;
    for (size_t i = 0; i < plan.size(); ++i) {
        const auto& p = plan[i];
        peers[i] = p.peer;
        send_counts[i] = (int)p.send.size() / 5;
        recv_counts[i] = (int)p.recv.size() / 5;
        std::copy(p.send.begin(), p.send.end(), records + 5 * k);
        k += send_counts[i];
        std::copy(p.recv.begin(), p.recv.end(), records + 5 * k);
        k += recv_counts[i];
    }
    return BMFR_OK;
}

bmfr_status bmfr_comm_unique_id(unsigned char id[128]) {
    if (!id) return BMFR_ERROR_INVALID_ARGUMENT;
    Rccl& r = rccl();
    if (!r.ok) return BMFR_ERROR_UNSUPPORTED;
    NcclId u;
    if (r.get_unique_id(&u) != 0) return BMFR_ERROR_HIP;
    std::memcpy(id, u.internal, sizeof(u.internal));
    return BMFR_OK;
}

bmfr_status bmfr_comm_create(const unsigned char id[128], int nranks, int rank, int hip_device, bmfr_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return BMFR_ERROR_INVALID_ARGUMENT;
    *out = nullptr;
    Rccl& r = rccl();
    if (!r.ok) return BMFR_ERROR_UNSUPPORTED;
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(hip_device) != hipSuccess) return BMFR_ERROR_NO_DEVICE;
    NcclId u;
    std::memcpy(u.internal, id, sizeof(u.internal));
    void* c = nullptr;
    const int e = r.comm_init_rank(&c, nranks, u, rank);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != 0) return BMFR_ERROR_HIP;
    *out = new bmfr_comm{c, nranks, rank, hip_device};
    return BMFR_OK;
}

bmfr_status bmfr_comm_create_all(int ndev, const int* devices, bmfr_comm** out) {
    if (ndev < 1 || !devices || !out) return BMFR_ERROR_INVALID_ARGUMENT;
    Rccl& r = rccl();
    if (!r.ok) return BMFR_ERROR_UNSUPPORTED;
    std::vector<void*> c(ndev, nullptr);
    if (r.comm_init_all(c.data(), ndev, devices) != 0) return BMFR_ERROR_HIP;
    for (int i = 0; i < ndev; ++i) out[i] = new bmfr_comm{c[i], ndev, i, devices[i]};
    return BMFR_OK;
}

bmfr_status bmfr_comm_destroy(bmfr_comm* comm) {
    if (!comm) return BMFR_ERROR_INVALID_ARGUMENT;
    if (comm->nccl) rccl().comm_destroy(comm->nccl);
    delete comm;
    return BMFR_OK;
}

bmfr_status bmfr_exchange_create(bmfr_ctx* ctx, const bmfr_config* cfg, const int* tiles, int ntiles, int rank,
                                 bmfr_comm* comm, bmfr_exchange** out) {
    if (!ctx || !out) return BMFR_ERROR_INVALID_ARGUMENT;
    *out = nullptr;
    bmfr_status s = validate_grid(cfg, tiles, ntiles, rank);
    if (s != BMFR_OK) return s;
    const int* t = tiles + 4 * rank;
    if (cfg->tile_x != t[0] || cfg->tile_y != t[1] || cfg->tile_width != t[2] || cfg->tile_height != t[3])
        return BMFR_ERROR_INVALID_ARGUMENT;  // cfg must be this rank's context configuration
    if (comm && (comm->nranks != ntiles || comm->rank != rank)) return BMFR_ERROR_INVALID_ARGUMENT;
    auto* x = new bmfr_exchange;
    x->ctx = ctx;
    x->comm = comm;
    x->rank = rank;
    x->ntiles = ntiles;
    for (int f = 0; f < 16; ++f) {
        if ((s = make_plan(cfg, tiles, ntiles, rank, f, x->plans[f])) != BMFR_OK) {
            delete x;
            return s;
        }
        for (auto& p : x->plans[f]) {
            // packed sizes (bmfr_halo_copy's layout); every message starts 16-byte aligned
            if (!p.send.empty() && (s = bmfr_halo_copy(ctx, nullptr, p.send.data(), (int)p.send.size() / 5,
                                                       nullptr, 0, &p.send_bytes)) != BMFR_OK)
                break;
            if (!p.recv.empty() && (s = bmfr_halo_copy(ctx, nullptr, p.recv.data(), (int)p.recv.size() / 5,
                                                       nullptr, 1, &p.recv_bytes)) != BMFR_OK)
                break;
            x->send_all[f].insert(x->send_all[f].end(), p.send.begin(), p.send.end());
            x->recv_all[f].insert(x->recv_all[f].end(), p.recv.begin(), p.recv.end());
            x->send_total[f] += p.send_bytes;
            x->recv_total[f] += p.recv_bytes;
        }
        if (s != BMFR_OK) {
            delete x;
            return s;
        }
        x->scap = std::max(x->scap, x->send_total[f]);
        x->rcap = std::max(x->rcap, x->recv_total[f]);
    }
    bmfr_sizes sz;
    (void)bmfr_get_sizes(ctx, &sz);
    int prev = -1;
    (void)hipGetDevice(&prev);
    // the context's device: the one whose memory bmfr_state points into
    bmfr_state_view v;
    (void)bmfr_state(ctx, 0, &v);
    hipPointerAttribute_t attr;
    x->device = hipPointerGetAttributes(&attr, v.result) == hipSuccess ? attr.device : (prev >= 0 ? prev : 0);
    if (comm && comm->device != x->device) {  // RCCL would move sbuf / rbuf of another GPU
        delete x;
        return BMFR_ERROR_INVALID_ARGUMENT;
    }
    (void)hipSetDevice(x->device);
    hipError_t e = hipSuccess;
    if (x->scap) e = hipMalloc(&x->sbuf, x->scap);
    if (e == hipSuccess && x->rcap) e = hipMalloc(&x->rbuf, x->rcap);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        (void)hipFree(x->sbuf);
        delete x;
        return BMFR_ERROR_OUT_OF_MEMORY;
    }
    *out = x;
    return BMFR_OK;
}

bmfr_status bmfr_exchange_destroy(bmfr_exchange* x) {
    if (!x) return BMFR_ERROR_INVALID_ARGUMENT;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(x->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(x->sbuf);
    (void)hipFree(x->rbuf);
    if (prev >= 0) (void)hipSetDevice(prev);
    delete x;
    return BMFR_OK;
}

bmfr_status bmfr_exchange_bytes(const bmfr_exchange* x, int frame_number, size_t* sent, size_t* received) {
    if (!x || frame_number < 0) return BMFR_ERROR_INVALID_ARGUMENT;
    if (sent) *sent = x->send_total[frame_number & 15];
    if (received) *received = x->recv_total[frame_number & 15];
    return BMFR_OK;
}

namespace {

// The RCCL part of one rank's exchange (inside a group the caller opened).
bmfr_status post_messages(bmfr_exchange* x, hipStream_t s, int f) {
    Rccl& r = rccl();
    size_t so = 0, ro = 0;
    for (const auto& p : x->plans[f]) {
        if (p.send_bytes && r.send(x->sbuf + so, p.send_bytes, kNcclUint8, p.peer, x->comm->nccl, s) != 0)
            return BMFR_ERROR_HIP;
        if (p.recv_bytes && r.recv(x->rbuf + ro, p.recv_bytes, kNcclUint8, p.peer, x->comm->nccl, s) != 0)
            return BMFR_ERROR_HIP;
        so += p.send_bytes;
        ro += p.recv_bytes;
    }
    return BMFR_OK;
}

bmfr_status pack(bmfr_exchange* x, hipStream_t s, int f) {
    const auto& v = x->send_all[f];
    return v.empty() ? BMFR_OK : bmfr_halo_copy(x->ctx, s, v.data(), (int)v.size() / 5, x->sbuf, 0, nullptr);
}

bmfr_status unpack(bmfr_exchange* x, hipStream_t s, int f) {
    const auto& v = x->recv_all[f];
    return v.empty() ? BMFR_OK : bmfr_halo_copy(x->ctx, s, v.data(), (int)v.size() / 5, x->rbuf, 1, nullptr);
}

}  // namespace

bmfr_status bmfr_exchange_run(bmfr_exchange* x, void* stream, int frame_number) {
    if (!x || frame_number < 0) return BMFR_ERROR_INVALID_ARGUMENT;
    if (!x->comm) return BMFR_ERROR_INVALID_ARGUMENT;  // in-process grids: bmfr_exchange_run_all
    const int f = frame_number & 15;
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    bmfr_status st = pack(x, s, f);
    if (st != BMFR_OK) return st;
    Rccl& r = rccl();
    if (r.group_start() != 0) return BMFR_ERROR_HIP;
    st = post_messages(x, s, f);
    if (r.group_end() != 0 && st == BMFR_OK) st = BMFR_ERROR_HIP;
    if (st != BMFR_OK) return st;
    return unpack(x, s, f);
}

bmfr_status bmfr_exchange_run_all(bmfr_exchange* const* xs, int n, void* const* streams, int frame_number) {
    if (!xs || n < 1 || !streams || frame_number < 0) return BMFR_ERROR_INVALID_ARGUMENT;
    for (int i = 0; i < n; ++i)
        if (!xs[i] || xs[i]->rank != i || xs[i]->ntiles != n || (xs[i]->comm == nullptr) != (xs[0]->comm == nullptr))
            return BMFR_ERROR_INVALID_ARGUMENT;
    const int f = frame_number & 15;
    bmfr_status st = BMFR_OK;
    if (xs[0]->comm) {
        // one process, one communicator per device (bmfr_comm_create_all): every
        // rank's messages in one group
        for (int i = 0; i < n && st == BMFR_OK; ++i) st = pack(xs[i], reinterpret_cast<hipStream_t>(streams[i]), f);
        if (st != BMFR_OK) return st;
        Rccl& r = rccl();
        if (r.group_start() != 0) return BMFR_ERROR_HIP;
        for (int i = 0; i < n && st == BMFR_OK; ++i)
            st = post_messages(xs[i], reinterpret_cast<hipStream_t>(streams[i]), f);
        if (r.group_end() != 0 && st == BMFR_OK) st = BMFR_ERROR_HIP;
        for (int i = 0; i < n && st == BMFR_OK; ++i) st = unpack(xs[i], reinterpret_cast<hipStream_t>(streams[i]), f);
        return st;
    }
    // No communicator: every context on one device, one stream (streams[0]).
    // The RCCL path's buffers exactly, with each ncclSend / ncclRecv pair
    // replaced by one device copy: every rank packs its send_all records into
    // its sbuf; each message then moves from the sender's sbuf (at the
    // sender's offset for that peer) into the receiver's rbuf (at the
    // receiver's offset for the sender); every rank unpacks its recv_all
    // records from its rbuf.  A message whose two ends disagree on its size is
    // a plan error (the RCCL receive would be truncated or wait forever).
    for (int i = 1; i < n; ++i)
        if (xs[i]->device != xs[0]->device) return BMFR_ERROR_UNSUPPORTED;
    // Both ends of every message are matched before anything is queued (a bad
    // plan is refused with nothing enqueued): (receiver, rbuf offset, sender,
    // sbuf offset, bytes) per message.
    struct Copy {
        int to, from;
        size_t ro, so, bytes;
    };
    std::vector<Copy> copies;
    for (int i = 0; i < n; ++i) {  // receiver i
        size_t ro = 0;
        for (const auto& p : xs[i]->plans[f]) {
            if (p.recv_bytes) {
                if (p.peer < 0 || p.peer >= n) return BMFR_ERROR_INVALID_ARGUMENT;
                const bmfr_exchange* y = xs[p.peer];  // the sender
                size_t so = 0;
                const PeerPlan* q = nullptr;
                for (const auto& yp : y->plans[f]) {
                    if (yp.peer == i) {
                        q = &yp;
                        break;
                    }
                    so += yp.send_bytes;
                }
                if (!q || q->send_bytes != p.recv_bytes || q->send != p.recv) return BMFR_ERROR_INVALID_ARGUMENT;
                copies.push_back({i, p.peer, ro, so, p.recv_bytes});
            }
            ro += p.recv_bytes;
        }
    }
    const hipStream_t s = reinterpret_cast<hipStream_t>(streams[0]);
    for (int i = 0; i < n && st == BMFR_OK; ++i) st = pack(xs[i], s, f);
    if (st != BMFR_OK) return st;
    for (const Copy& c : copies) {
        const hipError_t e =
            hipMemcpyAsync(xs[c.to]->rbuf + c.ro, xs[c.from]->sbuf + c.so, c.bytes, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return hip_st(e);
    }
    for (int i = 0; i < n && st == BMFR_OK; ++i) st = unpack(xs[i], s, f);
    return st;
}

}  // extern "C"
