// gic_multi.cpp -- multi-GPU encode from one host process behind the C ABI,
// and the lane driver shared with the host-image entry points.
//
// SURVEY.md 8(e) / north_star: "images shard by block-row across the GPUs of
// one node with a single RCCL gather of the packed BCn bitstream over xGMI at
// the end".  The reference's image wrappers walk every block row of every
// slice in one loop (amd_bc1_compressor.cpp:44-70, amd_bc7_compressor.cpp:
// 48-77); gic_encode_multi splits exactly that loop: the rows of all slices,
// numbered slice-major, are cut into one contiguous range per device, so each
// device's packed blocks form one contiguous piece of the reference-ordered
// output.  Per device (one host thread each, so BC7 calls -- which return with
// their device work complete, gic_bc7.hip H4 -- overlap across devices) the
// range runs through the upload / encode pipeline of gic_pipeline.cpp, and as
// soon as a device's last piece is encoded its blocks go to their offset in
// the root's buffer: ncclSend on the device's comm, matched by ncclRecv posted
// up front on a gather stream of the root (communicators from ncclCommInitAll
// over the list, built once per list), so the gather of a fast device overlaps
// the slower devices' encodes.  The root's own piece is encoded in place.  A
// list that names a device twice cannot form an RCCL communicator; it gathers
// with peer copies instead (the one-GPU test path of the same split).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "gfx_imagecompress_amd/gic.h"
#include "gic_pipeline.h"

namespace gic {

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int drive(std::vector<LaneJob> &jobs, const EncodeArgs &a, uint32_t bx, uint32_t by, ProgressFn cb, void *user)
{
    Progress prog;
    prog.done.assign(jobs.size(), 0);
    auto run = [&](int i) {
        LaneJob &j = jobs[i];
        const double t0 = now_ms();
        j.rc = run_pieces(*j.lane, a, j.pieces, &prog, i, &j.times);
        if (j.rc == GIC_OK && j.after && !prog.abort.load()) j.rc = j.after();
        j.wall_ms = now_ms() - t0;
        if (j.rc != GIC_OK) prog.abort.store(true);   // the other lanes stop between pieces
        prog.finish();
    };
    bool aborted = false;
    if (jobs.size() == 1 && !cb) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (size_t i = 0; i < jobs.size(); ++i) th.emplace_back(run, (int)i);
        if (cb) {
            // rows in slice-major order; row g belongs to the job whose range holds it
            uint64_t total = 0;
            for (const LaneJob &j : jobs) total = j.first_row + j.rows > total ? j.first_row + j.rows : total;
            size_t owner = 0;
            for (uint64_t g = 0; g < total && !aborted;) {
                while (owner < jobs.size() && g >= jobs[owner].first_row + jobs[owner].rows) ++owner;
                if (owner == jobs.size()) break;
                {
                    std::unique_lock<std::mutex> lk(prog.m);
                    prog.cv.wait(lk, [&] {
                        return g < jobs[owner].first_row + prog.done[owner] || prog.finished == (int)jobs.size();
                    });
                    if (g >= jobs[owner].first_row + prog.done[owner]) break;   // a lane failed
                }
                const uint64_t ready = jobs[owner].first_row + [&] {
                    std::lock_guard<std::mutex> lk(prog.m);
                    return prog.done[owner];
                }();
                for (; g < ready; ++g) {
                    const uint32_t y = (uint32_t)(g % by);
                    const float pct = 100.f * (y * bx) / (bx * by);
                    if (cb(user, pct)) {
                        aborted = true;
                        prog.abort.store(true);
                        break;
                    }
                }
            }
        }
        for (std::thread &t : th) t.join();
    }
    if (aborted) return GIC_EABORT;
    for (const LaneJob &j : jobs)
        if (j.rc != GIC_OK) return j.rc;
    return GIC_OK;
}

}  // namespace gic

namespace {

using Rank = gic::LaneBuffers;

struct Group {
    std::vector<int> devices;
    std::vector<std::unique_ptr<Rank>> ranks;
    std::vector<ncclComm_t> comms;   // empty: peer copies
    hipStream_t gather = nullptr;    // the root's receive stream (RCCL)
    bool rccl = false, tried = false;
};

std::mutex g_multi_lock;
Group g_group;
thread_local gic_multi_report t_report;

struct DeviceGuard {   // restores the caller's current device
    int dev = 0;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard() { (void)hipSetDevice(dev); }
};

void release(Group &g)
{
    for (ncclComm_t c : g.comms) (void)ncclCommDestroy(c);
    g.comms.clear();
    if (g.gather && !g.ranks.empty()) {
        (void)hipSetDevice(g.ranks[0]->lane.device);
        (void)hipStreamDestroy(g.gather);
    }
    g.gather = nullptr;
    for (auto &r : g.ranks) r->release();
    g.ranks.clear();
    g.devices.clear();
    g.rccl = g.tried = false;
}

// The group for this device list (caller holds g_multi_lock).
hipError_t get_group(int ndev, const int *devices, bool want_rccl, Group *&out)
{
    std::vector<int> want(devices, devices + ndev);
    if (g_group.devices != want) {
        release(g_group);
        g_group.devices = want;
        for (int i = 0; i < ndev; ++i) {
            g_group.ranks.emplace_back(new Rank);
            const hipError_t e = g_group.ranks.back()->lane.init(devices[i]);
            if (e != hipSuccess) {
                release(g_group);
                return e;
            }
        }
        hipError_t e = hipSetDevice(devices[0]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&g_group.gather, hipStreamNonBlocking);
        if (e != hipSuccess) {
            release(g_group);
            return e;
        }
    }
    bool distinct = true;
    for (int i = 0; i < ndev; ++i)
        for (int j = i + 1; j < ndev; ++j) distinct = distinct && devices[i] != devices[j];
    if (want_rccl && distinct && ndev > 1 && !g_group.tried) {
        g_group.tried = true;
        g_group.comms.resize(ndev);
        if (ncclCommInitAll(g_group.comms.data(), ndev, devices) == ncclSuccess) {
            g_group.rccl = true;
        } else {
            g_group.comms.clear();
            fprintf(stderr, "gfx_imagecompress_amd: ncclCommInitAll failed; gathering with peer copies\n");
        }
    }
    out = &g_group;
    return hipSuccess;
}

hipError_t grow(uint8_t *&p, size_t &cap, size_t need)
{
    if (need <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const hipError_t e = hipMalloc((void **)&p, need);
    if (e == hipSuccess) cap = need;
    return e;
}

bool valid_source(gic_source st) { return st == GIC_SRC_UNORM8 || st == GIC_SRC_SNORM8 || st == GIC_SRC_FLOAT32; }

}  // namespace

// contiguous ranges of the slice-major block rows, the first (rows % n) one longer
// (the same split as gfx_imagecompress_amd/shard.py shard_rows)
extern "C" int gic_multi_split(uint64_t rows_total, int ndev, int i, uint64_t *first, uint64_t *rows)
{
    if (ndev < 1 || i < 0 || i >= ndev || !first || !rows) return GIC_EINVAL;
    const uint64_t base = rows_total / ndev, extra = rows_total % ndev;
    *first = i * base + ((uint64_t)i < extra ? (uint64_t)i : extra);
    *rows = base + ((uint64_t)i < extra ? 1 : 0);
    return GIC_OK;
}

extern "C" int gic_encode_multi(gic_format fmt, gic_source src_type, const void *h_src, uint32_t width,
                                uint32_t height, uint32_t slices, uint32_t channels, size_t row_pitch,
                                const gic_options *opt, int ndev, const int *devices, uint8_t *d_dst_root,
                                uint32_t flags)
{
    if (!h_src || !d_dst_root || !width || !height || !slices || channels < 1 || channels > 4) return GIC_EINVAL;
    if (ndev < 1 || ndev > 64 || !devices || !valid_source(src_type)) return GIC_EINVAL;
    const size_t texel = (size_t)channels * (src_type == GIC_SRC_FLOAT32 ? 4 : 1);
    if (row_pitch < (size_t)width * texel) return GIC_EINVAL;
    const uint32_t bb = gic_block_bytes(fmt);
    if (!bb) return GIC_EINVAL;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return GIC_EHIP;
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= count) return GIC_EINVAL;
    const uint32_t bx = (width + 3) / 4, by = (height + 3) / 4;
    const uint64_t rows_total = (uint64_t)by * slices;
    const size_t row_bytes = (size_t)bx * bb;   // packed blocks of one block row

    std::lock_guard<std::mutex> lk(g_multi_lock);
    DeviceGuard guard;
    Group *g = nullptr;
    if (get_group(ndev, devices, !(flags & GIC_MULTI_PEER_COPY), g) != hipSuccess) return GIC_EHIP;
    const bool rccl = g->rccl && !(flags & GIC_MULTI_PEER_COPY);
    t_report = gic_multi_report{};
    t_report.ranks = ndev;
    t_report.rccl = rccl ? 1 : 0;

    const gic::EncodeArgs args{fmt, src_type, width, height, channels, row_pitch, opt};
    std::vector<gic::LaneJob> jobs(ndev);
    std::vector<double> encoded_at(ndev, 0.0);
    const double t0 = gic::now_ms();
    for (int i = 0; i < ndev; ++i) {
        Rank &r = *g->ranks[i];
        uint64_t first = 0, n = 0;
        gic_multi_split(rows_total, ndev, i, &first, &n);
        gic::LaneJob &j = jobs[i];
        j.lane = &r.lane;
        j.first_row = first;
        j.rows = n;
        if (!n) continue;
        if (hipSetDevice(r.lane.device) != hipSuccess) return GIC_EHIP;
        if (grow(r.src, r.src_cap, gic::slab_bytes(first, n, by, height, row_pitch)) != hipSuccess) return GIC_EHIP;
        if (i && grow(r.dst, r.dst_cap, n * row_bytes) != hipSuccess) return GIC_EHIP;
        uint8_t *out = i ? r.dst : d_dst_root + first * row_bytes;
        j.pieces = gic::make_pieces(first, n, gic::piece_plan(fmt, bx, n), by, height, row_pitch, row_bytes, (const uint8_t *)h_src, r.src,
                                    out, nullptr);
        if (!i) {
            j.after = [&, i] {
                encoded_at[i] = gic::now_ms();
                return GIC_OK;
            };
            continue;
        }
        // the device's blocks go to the root as soon as its last piece is encoded
        j.after = [&, i, first, n] {
            Rank &rr = *g->ranks[i];
            encoded_at[i] = gic::now_ms();
            const size_t bytes = n * row_bytes;
            hipError_t e = hipSuccess;
            if (rccl) {
                const ncclResult_t nr = ncclSend(rr.dst, bytes, ncclUint8, 0, g->comms[i], rr.lane.enc);
                if (nr != ncclSuccess) {
                    fprintf(stderr, "gfx_imagecompress_amd: RCCL send failed (%s)\n", ncclGetErrorString(nr));
                    return GIC_EHIP;
                }
            } else {
                e = hipMemcpyPeerAsync(d_dst_root + first * row_bytes, g->ranks[0]->lane.device, rr.dst,
                                       rr.lane.device, bytes, rr.lane.enc);
            }
            if (e == hipSuccess) e = hipStreamSynchronize(rr.lane.enc);
            return e == hipSuccess ? GIC_OK : GIC_EHIP;
        };
    }
    // RCCL: the root's receives are posted up front on its gather stream, in
    // rank order, before the senders start (each pair has one send / recv)
    std::thread receiver;
    int recv_rc = GIC_OK;
    if (rccl) {
        receiver = std::thread([&] {
            (void)hipSetDevice(g->ranks[0]->lane.device);
            for (int i = 1; i < ndev && recv_rc == GIC_OK; ++i) {
                if (!jobs[i].rows) continue;
                const ncclResult_t nr = ncclRecv(d_dst_root + jobs[i].first_row * row_bytes, jobs[i].rows * row_bytes,
                                                 ncclUint8, i, g->comms[0], g->gather);
                if (nr != ncclSuccess) {
                    fprintf(stderr, "gfx_imagecompress_amd: RCCL receive failed (%s)\n", ncclGetErrorString(nr));
                    recv_rc = GIC_EHIP;
                }
            }
            if (recv_rc == GIC_OK && hipStreamSynchronize(g->gather) != hipSuccess) recv_rc = GIC_EHIP;
        });
    }
    int rc = gic::drive(jobs, args, bx, by, nullptr, nullptr);
    if (rc != GIC_OK && rccl) {
        // a device failed before its send: the root's posted receive would wait
        // forever, so the communicators are aborted (rebuilt by the next call)
        for (ncclComm_t c : g->comms) (void)ncclCommAbort(c);
        g->comms.clear();
        g->rccl = g->tried = false;
    }
    if (receiver.joinable()) receiver.join();
    const double t1 = gic::now_ms();
    if (rc == GIC_OK) rc = recv_rc;
    if (rc != GIC_OK) return rc;
    double last_encoded = 0.0;
    for (int i = 0; i < ndev; ++i) {
        if (!jobs[i].rows) continue;
        const double enc = encoded_at[i] - t0;
        t_report.encode_ms_max = enc > t_report.encode_ms_max ? enc : t_report.encode_ms_max;
        last_encoded = encoded_at[i] > last_encoded ? encoded_at[i] : last_encoded;
        if (i) t_report.gathered_bytes += jobs[i].rows * row_bytes;
    }
    // the gather's exposed part: from the last device's encode to the end of the call
    t_report.gather_ms = t1 - last_encoded > 0 ? t1 - last_encoded : 0.0;
    return GIC_OK;
}

namespace gic {

hipError_t LaneBuffers::reserve(size_t src_bytes, size_t dst_bytes)
{
    hipError_t e = hipSetDevice(lane.device);
    if (e == hipSuccess) e = grow(src, src_cap, src_bytes);
    if (e == hipSuccess) e = grow(dst, dst_cap, dst_bytes);
    return e;
}

void LaneBuffers::release()
{
    if (lane.device >= 0) {
        (void)hipSetDevice(lane.device);
        if (src) (void)hipFree(src);
        if (dst) (void)hipFree(dst);
    }
    src = dst = nullptr;
    src_cap = dst_cap = 0;
    lane.release();
}

int encode_host(const std::vector<LaneBuffers *> &lanes, const EncodeArgs &a, const uint8_t *h_src, uint32_t slices,
                uint8_t *h_out, ProgressFn cb, void *user, gic_host_report *rep)
{
    const double t0 = now_ms();
    const uint32_t bb = gic_block_bytes(a.fmt);
    const uint32_t bx = (a.width + 3) / 4, by = (a.height + 3) / 4;
    const uint64_t rows_total = (uint64_t)by * slices;
    const size_t row_bytes = (size_t)bx * bb;
    const int n = (int)lanes.size();
    std::vector<LaneJob> jobs(n);
    for (int i = 0; i < n; ++i) {
        uint64_t first = 0, rows = 0;
        gic_multi_split(rows_total, n, i, &first, &rows);
        LaneJob &j = jobs[i];
        j.lane = &lanes[i]->lane;
        j.first_row = first;
        j.rows = rows;
        if (!rows) continue;
        if (lanes[i]->reserve(slab_bytes(first, rows, by, a.height, a.row_pitch), rows * row_bytes) != hipSuccess)
            return GIC_EHIP;
        j.pieces = make_pieces(first, rows, piece_plan(a.fmt, bx, rows), by, a.height, a.row_pitch, row_bytes, h_src, lanes[i]->src,
                               lanes[i]->dst, h_out + first * row_bytes);
    }
    const int rc = drive(jobs, a, bx, by, cb, user);
    if (rep) {
        *rep = gic_host_report{};
        rep->devices = n;
        rep->h2d_mode = (int)h2d_mode();
        rep->total_ms = now_ms() - t0;
        for (const LaneJob &j : jobs) {
            rep->pieces += (int)j.pieces.size();
            rep->h2d_ms = j.times.h2d_ms > rep->h2d_ms ? j.times.h2d_ms : rep->h2d_ms;
            rep->encode_ms = j.times.encode_ms > rep->encode_ms ? j.times.encode_ms : rep->encode_ms;
            rep->d2h_ms = j.times.d2h_ms > rep->d2h_ms ? j.times.d2h_ms : rep->d2h_ms;
        }
    }
    return rc;
}

int encode_host_devices(const std::vector<int> &devices, const EncodeArgs &a, const uint8_t *h_src, uint32_t slices,
                        uint8_t *h_out, ProgressFn cb, void *user, gic_host_report *rep)
{
    std::lock_guard<std::mutex> lk(g_multi_lock);
    DeviceGuard guard;
    Group *g = nullptr;
    if (get_group((int)devices.size(), devices.data(), false, g) != hipSuccess) return GIC_EHIP;
    std::vector<LaneBuffers *> lanes;
    for (auto &r : g->ranks) lanes.push_back(r.get());
    return encode_host(lanes, a, h_src, slices, h_out, cb, user, rep);
}

}  // namespace gic

extern "C" int gic_multi_last_report(gic_multi_report *out)
{
    if (!out) return GIC_EINVAL;
    *out = t_report;
    return GIC_OK;
}

extern "C" int gic_multi_release(void)
{
    std::lock_guard<std::mutex> lk(g_multi_lock);
    DeviceGuard guard;
    release(g_group);
    return GIC_OK;
}
