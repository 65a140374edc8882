// gic_multi.cpp -- multi-GPU encode from one host process behind the C ABI.
//
// SURVEY.md 8(e) / north_star: "images shard by block-row across the GPUs of
// one node with a single RCCL gather of the packed BCn bitstream over xGMI at
// the end".  The reference's image wrappers walk every block row of every
// slice in one loop (amd_bc1_compressor.cpp:44-70, amd_bc7_compressor.cpp:
// 48-77); gic_encode_multi splits exactly that loop: the rows of all slices,
// numbered slice-major, are cut into one contiguous range per device, so each
// device's packed blocks form one contiguous piece of the reference-ordered
// output.  Per device (one host thread each, so BC7 calls -- which return with
// their device work complete, gic_bc7.hip H4 -- overlap across devices):
// upload the source rows its range reads, encode them with the row-range entry
// (gic_hip_encode_rows_src) on its own stream.  Then one gather: grouped
// ncclSend / ncclRecv over communicators from ncclCommInitAll (built once per
// device list) lands every piece at its offset in the root's buffer; the root's
// own piece is encoded in place.  A list that names a device twice cannot form
// an RCCL communicator; it gathers with peer copies instead (the one-GPU test
// path of the same split).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "gfx_imagecompress_amd/gic.h"

namespace {

struct Rank {
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t *src = nullptr, *dst = nullptr;
    size_t src_cap = 0, dst_cap = 0;
};

struct Group {
    std::vector<int> devices;
    std::vector<Rank> ranks;
    std::vector<ncclComm_t> comms;   // empty: peer copies
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
    for (Rank &r : g.ranks) {
        if (r.device < 0) continue;
        (void)hipSetDevice(r.device);
        if (r.src) (void)hipFree(r.src);
        if (r.dst) (void)hipFree(r.dst);
        if (r.done) (void)hipEventDestroy(r.done);
        if (r.stream) (void)hipStreamDestroy(r.stream);
    }
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
        g_group.ranks.resize(ndev);
        for (int i = 0; i < ndev; ++i) {
            Rank &r = g_group.ranks[i];
            r.device = devices[i];
            hipError_t e = hipSetDevice(r.device);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&r.done, hipEventDisableTiming);
            if (e != hipSuccess) {
                release(g_group);
                return e;
            }
        }
    }
    bool distinct = true;
    for (int i = 0; i < ndev; ++i)
        for (int j = i + 1; j < ndev; ++j) distinct = distinct && devices[i] != devices[j];
    if (want_rccl && distinct && ndev > 1 && !g_group.tried) {
        g_group.tried = true;
        {
            g_group.comms.resize(ndev);
            if (ncclCommInitAll(g_group.comms.data(), ndev, devices) == ncclSuccess) {
                g_group.rccl = true;
            } else {
                g_group.comms.clear();
                fprintf(stderr, "gfx_imagecompress_amd: ncclCommInitAll failed; gathering with peer copies\n");
            }
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
    if (ndev < 1 || ndev > 64 || !devices) return GIC_EINVAL;
    if (src_type != GIC_SRC_UNORM8 && src_type != GIC_SRC_SNORM8 && src_type != GIC_SRC_FLOAT32) return GIC_EINVAL;
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
    const size_t slice_bytes = row_pitch * height;

    std::lock_guard<std::mutex> lk(g_multi_lock);
    DeviceGuard guard;
    Group *g = nullptr;
    hipError_t e = get_group(ndev, devices, !(flags & GIC_MULTI_PEER_COPY), g);
    if (e != hipSuccess) return GIC_EHIP;
    const bool rccl = g->rccl && !(flags & GIC_MULTI_PEER_COPY);

    std::vector<uint64_t> first(ndev), nrows(ndev);
    for (int i = 0; i < ndev; ++i) gic_multi_split(rows_total, ndev, i, &first[i], &nrows[i]);
    t_report = gic_multi_report{};
    t_report.ranks = ndev;
    t_report.rccl = rccl ? 1 : 0;

    std::vector<int> rc(ndev, GIC_OK);
    std::vector<hipError_t> he(ndev, hipSuccess);
    std::vector<double> enc_ms(ndev, 0.0);
    auto encode_rank = [&](int i) {
        Rank &r = g->ranks[i];
        hipError_t err = hipSetDevice(r.device);
        if (err != hipSuccess || !nrows[i]) {
            he[i] = err;
            return;
        }
        // the slice segments of the range and the source bytes they read
        struct Seg {
            uint32_t slice, y0, y1;
            size_t off;   // into the rank's source slab
        };
        std::vector<Seg> segs;
        size_t slab = 0;
        for (uint64_t row = first[i], end = first[i] + nrows[i]; row < end;) {
            const uint32_t w = (uint32_t)(row / by), y0 = (uint32_t)(row % by);
            const uint32_t y1 = (uint32_t)((end - (uint64_t)w * by) < by ? (end - (uint64_t)w * by) : by);
            const uint32_t py1 = 4 * y1 < height ? 4 * y1 : height;
            segs.push_back({w, y0, y1, slab});
            slab += (size_t)(py1 - 4 * y0) * row_pitch;
            row = (uint64_t)w * by + y1;
        }
        const bool root = i == 0;
        err = grow(r.src, r.src_cap, slab);
        if (err == hipSuccess && !root) err = grow(r.dst, r.dst_cap, nrows[i] * row_bytes);
        hipEvent_t t0 = nullptr, t1 = nullptr;
        if (err == hipSuccess) err = hipEventCreate(&t0);
        if (err == hipSuccess) err = hipEventCreate(&t1);
        if (err == hipSuccess) err = hipEventRecord(t0, r.stream);
        for (const Seg &sg : segs) {
            if (err != hipSuccess) break;
            const uint32_t py1 = 4 * sg.y1 < height ? 4 * sg.y1 : height;
            const uint8_t *hs = (const uint8_t *)h_src + slice_bytes * sg.slice + (size_t)4 * sg.y0 * row_pitch;
            err = hipMemcpyAsync(r.src + sg.off, hs, (size_t)(py1 - 4 * sg.y0) * row_pitch, hipMemcpyHostToDevice,
                                 r.stream);
        }
        size_t out_off = 0;
        for (const Seg &sg : segs) {
            if (err != hipSuccess) break;
            // the slab holds pixel rows [4 y0, ...) of the slice: address it as the
            // whole slice (the kernels read only rows of block rows y0..y1-1, and
            // the edge clamp of the image's last block row stays inside the slab)
            const uint8_t *base = r.src + sg.off - (size_t)4 * sg.y0 * row_pitch;
            uint8_t *out = root ? d_dst_root + first[i] * row_bytes + out_off : r.dst + out_off;
            rc[i] = gic_hip_encode_rows_src(fmt, src_type, base, width, height, 1, channels, row_pitch, sg.y0,
                                            sg.y1 - sg.y0, opt, out, nullptr, r.stream);
            if (rc[i] != GIC_OK) break;
            out_off += (size_t)(sg.y1 - sg.y0) * row_bytes;
        }
        if (err == hipSuccess) err = hipEventRecord(t1, r.stream);
        if (err == hipSuccess) err = hipEventRecord(r.done, r.stream);
        if (err == hipSuccess) err = hipStreamSynchronize(r.stream);
        float ms = 0.f;
        if (err == hipSuccess && hipEventElapsedTime(&ms, t0, t1) == hipSuccess) enc_ms[i] = ms;
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
        he[i] = err;
    };
    {
        std::vector<std::thread> th;
        for (int i = 1; i < ndev; ++i) th.emplace_back(encode_rank, i);
        encode_rank(0);
        for (std::thread &t : th) t.join();
    }
    for (int i = 0; i < ndev; ++i) {
        if (rc[i] != GIC_OK) return rc[i];
        if (he[i] != hipSuccess) return GIC_EHIP;
        t_report.encode_ms_max = enc_ms[i] > t_report.encode_ms_max ? enc_ms[i] : t_report.encode_ms_max;
    }

    // the gather: every non-root piece to its offset in the root's buffer
    Rank &root = g->ranks[0];
    hipEvent_t g0 = nullptr, g1 = nullptr;
    e = hipSetDevice(root.device);
    if (e == hipSuccess) e = hipEventCreate(&g0);
    if (e == hipSuccess) e = hipEventCreate(&g1);
    if (e == hipSuccess) e = hipEventRecord(g0, root.stream);
    if (e != hipSuccess) return GIC_EHIP;
    if (rccl) {
        ncclResult_t nr = ncclGroupStart();
        for (int i = 1; i < ndev && nr == ncclSuccess; ++i) {
            if (!nrows[i]) continue;
            const size_t n = nrows[i] * row_bytes;
            nr = ncclSend(g->ranks[i].dst, n, ncclUint8, 0, g->comms[i], g->ranks[i].stream);
            if (nr == ncclSuccess)
                nr = ncclRecv(d_dst_root + first[i] * row_bytes, n, ncclUint8, i, g->comms[0], root.stream);
        }
        const ncclResult_t ne = ncclGroupEnd();
        if (nr != ncclSuccess || ne != ncclSuccess) {
            fprintf(stderr, "gfx_imagecompress_amd: RCCL gather failed (%s)\n",
                    ncclGetErrorString(nr != ncclSuccess ? nr : ne));
            return GIC_EHIP;
        }
    } else {
        for (int i = 1; i < ndev && e == hipSuccess; ++i) {
            if (!nrows[i]) continue;
            const size_t n = nrows[i] * row_bytes;
            e = hipMemcpyPeerAsync(d_dst_root + first[i] * row_bytes, root.device, g->ranks[i].dst,
                                   g->ranks[i].device, n, root.stream);
        }
    }
    if (e == hipSuccess) e = hipEventRecord(g1, root.stream);
    for (int i = 0; i < ndev && e == hipSuccess; ++i) {
        e = hipSetDevice(g->ranks[i].device);
        if (e == hipSuccess) e = hipStreamSynchronize(g->ranks[i].stream);
    }
    float gms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&gms, g0, g1);
    (void)hipSetDevice(root.device);
    (void)hipEventDestroy(g0);
    (void)hipEventDestroy(g1);
    if (e != hipSuccess) return GIC_EHIP;
    t_report.gather_ms = gms;
    for (int i = 1; i < ndev; ++i) t_report.gathered_bytes += nrows[i] * row_bytes;
    return GIC_OK;
}

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
