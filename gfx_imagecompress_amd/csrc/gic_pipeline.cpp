// gic_pipeline.cpp -- upload / encode / download overlap for host images
// (see gic_pipeline.h).
#include "gic_pipeline.h"

#include <sys/mman.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23   // Linux 5.14
#endif

namespace gic {

void *alloc_image_data(size_t bytes)
{
    constexpr size_t kHuge = (size_t)2 << 20;
    if (bytes < 2 * kHuge) return malloc(bytes ? bytes : 1);
    void *p = nullptr;
    if (posix_memalign(&p, kHuge, bytes) != 0) return nullptr;
    (void)madvise(p, (bytes + kHuge - 1) & ~(kHuge - 1), MADV_HUGEPAGE);   // a hint: ignored where THP is off
    return p;
}

// Faults in the pages of [p, p + bytes) for writing without touching their
// contents (so it may run beside threads writing the same range); a no-op on
// kernels without MADV_POPULATE_WRITE.
static void populate_write(void *p, size_t bytes)
{
    static const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = (uintptr_t)p & ~(page - 1), b = ((uintptr_t)p + bytes + page - 1) & ~(page - 1);
    if (b > a) (void)madvise((void *)a, b - a, MADV_POPULATE_WRITE);
}

H2D h2d_mode()
{
    const char *e = getenv("GIC_H2D");   // read per call: a process may compare modes
    if (!e || !*e || !strcmp(e, "pageable")) return H2D::Pageable;
    if (!strcmp(e, "staged")) return H2D::Staged;
    if (!strcmp(e, "register")) return H2D::Register;
    static std::once_flag warned;
    std::call_once(warned, [e] {
        fprintf(stderr, "gfx_imagecompress_amd: GIC_H2D=%s not understood (pageable | staged | register); "
                        "using pageable\n", e);
    });
    return H2D::Pageable;
}

static constexpr int kStageSlots = 3;

hipError_t Lane::init(int dev)
{
    if (device == dev && up) return hipSuccess;
    release();
    device = dev;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&up, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&enc, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&enc2, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&enc3, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&down, hipStreamNonBlocking);
    for (hipEvent_t *t : {&t_up0, &t_up1, &t_enc0, &t_enc1})
        if (e == hipSuccess) e = hipEventCreate(t);
    if (e != hipSuccess) release();
    return e;
}

hipError_t Lane::reserve_events(size_t pieces)
{
    hipError_t e = hipSuccess;
    while (e == hipSuccess && ev_up.size() < pieces) {
        hipEvent_t a = nullptr, b = nullptr;
        e = hipEventCreateWithFlags(&a, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&b, hipEventDisableTiming);
        if (e != hipSuccess) {
            if (a) (void)hipEventDestroy(a);
            break;
        }
        ev_up.push_back(a);
        ev_enc.push_back(b);
    }
    return e;
}

hipError_t Lane::reserve_zc(size_t bytes, bool non_coherent)
{
    if (bytes <= zc_cap && non_coherent == zc_nc) return hipSuccess;
    if (zc) (void)hipHostFree(zc);
    zc = nullptr;
    zc_cap = 0;
    const hipError_t e =
        hipHostMalloc((void **)&zc, bytes, non_coherent ? hipHostMallocNonCoherent : hipHostMallocDefault);
    if (e == hipSuccess) {
        zc_cap = bytes;
        zc_nc = non_coherent;
    }
    return e;
}

hipError_t Lane::reserve_stage(size_t slot_bytes)
{
    if (slot_bytes <= stage_slot) return hipSuccess;
    if (stage) (void)hipHostFree(stage);
    stage = nullptr;
    stage_slot = 0;
    const hipError_t e = hipHostMalloc((void **)&stage, slot_bytes * kStageSlots, hipHostMallocDefault);
    if (e == hipSuccess) stage_slot = slot_bytes;
    return e;
}

void Lane::release()
{
    if (device >= 0) (void)hipSetDevice(device);
    for (hipEvent_t ev : ev_up) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : ev_enc) (void)hipEventDestroy(ev);
    ev_up.clear();
    ev_enc.clear();
    for (hipEvent_t *t : {&t_up0, &t_up1, &t_enc0, &t_enc1}) {
        if (*t) (void)hipEventDestroy(*t);
        *t = nullptr;
    }
    for (hipStream_t *s : {&up, &enc, &enc2, &enc3, &down}) {
        if (*s) (void)hipStreamDestroy(*s);
        *s = nullptr;
    }
    if (stage) (void)hipHostFree(stage);
    stage = nullptr;
    stage_slot = 0;
    if (zc) (void)hipHostFree(zc);
    zc = nullptr;
    zc_cap = 0;
    device = -1;
}

PiecePlan piece_plan(gic_format fmt, uint32_t blocks_x, uint64_t rows)
{
    const uint64_t bx = blocks_x ? blocks_x : 1;
    auto clamp_rows = [](uint64_t r) { return r < 1 ? 1u : (r > 0xffffffffull ? 0xffffffffu : (uint32_t)r); };
    const char *e = getenv("GIC_PIECE_BLOCKS");   // test / tuning hooks
    const char *f = getenv("GIC_PIECE_FIRST");
    if (e && atoll(e) > 0) {
        const uint32_t r = clamp_rows((uint64_t)atoll(e) / bx);
        return PiecePlan{f && atoll(f) > 0 ? clamp_rows((uint64_t)atoll(f) / bx) : r, r};
    }
    if (fmt == GIC_FMT_BC7) return PiecePlan{clamp_rows(rows / 16), 0xffffffffu};
    const uint32_t r = clamp_rows((1u << 18) / bx);
    return PiecePlan{r, r};
}

size_t slab_bytes(uint64_t first, uint64_t rows, uint32_t by, uint32_t height, size_t pitch)
{
    size_t bytes = 0;
    for (uint64_t row = first, end = first + rows; row < end;) {
        const uint64_t w = row / by;
        const uint32_t y0 = (uint32_t)(row % by);
        const uint64_t y1 = (end - w * by) < by ? (end - w * by) : by;
        const uint32_t py1 = 4 * y1 < height ? (uint32_t)(4 * y1) : height;
        bytes += (size_t)(py1 - 4 * y0) * pitch;
        row = w * by + y1;
    }
    return bytes;
}

std::vector<Piece> make_pieces(uint64_t first, uint64_t rows, const PiecePlan &plan, uint32_t by, uint32_t height,
                               size_t pitch, size_t row_bytes, const uint8_t *h_src, uint8_t *d_slab, uint8_t *d_out,
                               uint8_t *h_out)
{
    std::vector<Piece> out;
    const size_t slice_bytes = pitch * height;
    size_t off = 0;
    for (uint64_t row = first, end = first + rows; row < end;) {
        const uint32_t w = (uint32_t)(row / by), y0 = (uint32_t)(row % by);
        uint64_t n = by - y0;
        const uint32_t per = out.empty() ? plan.first : plan.per;
        if (n > per) n = per;
        if (n > end - row) n = end - row;
        const uint32_t py1 = 4 * (y0 + n) < height ? (uint32_t)(4 * (y0 + n)) : height;
        Piece p;
        p.slice = w;
        p.y0 = y0;
        p.n = (uint32_t)n;
        p.h_src = h_src + slice_bytes * w + (size_t)4 * y0 * pitch;
        p.src_bytes = (size_t)(py1 - 4 * y0) * pitch;
        p.d_src = d_slab + off;
        // the slab holds pixel rows [4 y0, py1) of the slice here: address it as
        // the whole slice (the kernels read only the rows of block rows y0..y0+n-1,
        // and the last block row's edge clamp stays inside them)
        p.d_slice = p.d_src - (size_t)4 * y0 * pitch;
        p.d_out = d_out + (row - first) * row_bytes;
        p.h_out = h_out ? h_out + (row - first) * row_bytes : nullptr;
        p.out_bytes = n * row_bytes;
        out.push_back(p);
        off += p.src_bytes;
        row += n;
    }
    return out;
}

namespace {

// A counter one stage raises and the next waits on.
struct Handoff {
    std::mutex m;
    std::condition_variable cv;
    size_t ready = 0;
    bool failed = false;
    void post(size_t k)
    {
        {
            std::lock_guard<std::mutex> lk(m);
            ready = k;
        }
        cv.notify_all();
    }
    void fail()
    {
        {
            std::lock_guard<std::mutex> lk(m);
            failed = true;
        }
        cv.notify_all();
    }
    // true once piece k is ready; false if the producer failed or stopped first
    bool wait(size_t k)
    {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return ready > k || failed; });
        return ready > k;
    }
};

struct Registration {   // page-locks a host range for the call (H2D::Register)
    void *base = nullptr;
    hipError_t lock(const void *p, size_t bytes)
    {
        const uintptr_t page = 4096, a = (uintptr_t)p & ~(page - 1);
        const size_t len = (((uintptr_t)p + bytes + page - 1) & ~(page - 1)) - a;
        const hipError_t e = hipHostRegister((void *)a, len, hipHostRegisterDefault);
        if (e == hipSuccess) base = (void *)a;
        return e;
    }
    ~Registration()
    {
        if (base) (void)hipHostUnregister(base);
    }
};

float span_ms(hipEvent_t a, hipEvent_t b)
{
    float ms = 0.f;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

}  // namespace

int run_pieces(Lane &lane, const EncodeArgs &a, const std::vector<Piece> &pieces, Progress *progress, int lane_index,
               StageTimes *times)
{
    if (pieces.empty()) return GIC_OK;
    hipError_t e = hipSetDevice(lane.device);
    if (e == hipSuccess) e = lane.reserve_events(pieces.size());
    const H2D mode = h2d_mode();
    size_t max_src = 0;
    for (const Piece &p : pieces) max_src = p.src_bytes > max_src ? p.src_bytes : max_src;
    if (e == hipSuccess && mode == H2D::Staged) e = lane.reserve_stage(max_src);
    // zero-copy outputs (see the download stage): piece k at zc + zc_off[k]
    std::vector<size_t> zc_off(pieces.size(), 0);
    size_t zc_bytes = 0;
    for (size_t k = 0; k < pieces.size(); ++k) {
        zc_off[k] = zc_bytes;
        if (pieces[k].h_out) zc_bytes += pieces[k].out_bytes;
    }
    // GIC_PIPE_ZC_NC=1 (tuning hook): the kernels' host-image outputs in
    // non-coherent (coarse-grained) pinned memory, made visible at each kernel's end
    const char *zc_env = getenv("GIC_PIPE_ZC_NC");
    if (e == hipSuccess && zc_bytes) e = lane.reserve_zc(zc_bytes, zc_env && atoi(zc_env) > 0);
    double d2h_span = 0;
    Registration reg;
    if (e == hipSuccess && mode == H2D::Register) {
        // pieces of one lane read one contiguous host range (slices are stacked)
        const uint8_t *lo = pieces.front().h_src, *hi = pieces.back().h_src + pieces.back().src_bytes;
        e = reg.lock(lo, (size_t)(hi - lo));
    }
    if (e != hipSuccess) return GIC_EHIP;

    // tuning / diagnosis hooks (read per call): GIC_PIPE_POLL=1 the copy-out
    // stage polls hipEventQuery instead of blocking in hipEventSynchronize;
    // GIC_PIPE_INLINE_UP=1 (register mode) the encoding thread enqueues each
    // piece's upload itself, no upload thread; GIC_PIPE_NOPOP=1 no page
    // populating; GIC_PIPE_NOCOPY=1 no copy into the caller's image (timing only:
    // the image is left unwritten)
    auto flag = [](const char *n) { const char *v = getenv(n); return v && atoi(v) > 0; };
    const bool poll = flag("GIC_PIPE_POLL"), inline_up = flag("GIC_PIPE_INLINE_UP") && mode == H2D::Register,
               no_pop = flag("GIC_PIPE_NOPOP"), no_copy = flag("GIC_PIPE_NOCOPY");
    Handoff uploaded, encoded;
    hipError_t e_up = hipSuccess, e_dn = hipSuccess;
    std::atomic<bool> halt{false};   // the encoder failed: the other stages stop too
    auto stop = [&] { return halt.load() || (progress && progress->abort.load(std::memory_order_relaxed)); };

    std::thread uploader([&] {
        if (inline_up) return;
        hipError_t err = hipSetDevice(lane.device);
        if (err == hipSuccess) err = hipEventRecord(lane.t_up0, lane.up);
        for (size_t k = 0; k < pieces.size() && err == hipSuccess && !stop(); ++k) {
            const Piece &p = pieces[k];
            if (mode == H2D::Staged) {
                // slot k % kStageSlots was last DMAed by piece k - kStageSlots
                if (k >= (size_t)kStageSlots) err = hipEventSynchronize(lane.ev_up[k - kStageSlots]);
                uint8_t *slot = lane.stage + (k % kStageSlots) * lane.stage_slot;
                if (err == hipSuccess) {
                    memcpy(slot, p.h_src, p.src_bytes);
                    err = hipMemcpyAsync(p.d_src, slot, p.src_bytes, hipMemcpyHostToDevice, lane.up);
                }
            } else {
                err = hipMemcpyAsync(p.d_src, p.h_src, p.src_bytes, hipMemcpyHostToDevice, lane.up);
            }
            if (err == hipSuccess) err = hipEventRecord(lane.ev_up[k], lane.up);
            if (err == hipSuccess) uploaded.post(k + 1);
        }
        if (err == hipSuccess) err = hipEventRecord(lane.t_up1, lane.up);
        e_up = err;
        uploaded.fail();   // wakes the encoder if it waits past the last posted piece
    });

    // The caller's image pages are faulted in ahead of the copy-out stage, in
    // piece order (a fresh allocation faults on first touch: several ms for an
    // 8K BC1 image if the copies took them one by one).
    std::thread populator([&] {
        for (size_t k = 0; k < pieces.size() && !stop() && !no_pop; ++k)
            if (pieces[k].h_out) populate_write(pieces[k].h_out, pieces[k].out_bytes);
    });

    // Pieces with a host destination are encoded straight into pinned host
    // memory (the kernels' block stores cross PCIe as they retire), and the
    // download stage only copies each finished piece into the caller's image.
    // A device-to-host copy would be a blit kernel, and that waits for free CUs
    // -- behind every queued encode kernel, i.e. after the last one (rocprofv3
    // trace of round 6, profiles/r06_host_pipeline_trace.txt).
    std::thread downloader([&] {
        hipError_t err = hipSetDevice(lane.device);
        double t0 = 0, t1 = 0;
        for (size_t k = 0; k < pieces.size() && err == hipSuccess; ++k) {
            if (!encoded.wait(k)) break;
            const Piece &p = pieces[k];
            if (poll) {
                while ((err = hipEventQuery(lane.ev_enc[k])) == hipErrorNotReady)
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
            } else {
                err = hipEventSynchronize(lane.ev_enc[k]);
            }
            if (err == hipSuccess && p.h_out) {
                const double t = now_ms();
                if (t0 == 0) t0 = t;
                if (!no_copy) memcpy(p.h_out, lane.zc + zc_off[k], p.out_bytes);
                t1 = now_ms();
            }
            if (err == hipSuccess && progress) progress->add(lane_index, p.n);
        }
        d2h_span = t1 - t0;
        e_dn = err;
    });

    // consecutive pieces alternate between the lane's encode streams, two by
    // default (BC7 calls complete before they return, so BC7 keeps one);
    // GIC_ENC_STREAMS (1-3) is a tuning hook
    const char *es_env = getenv("GIC_ENC_STREAMS");   // read per call, like GIC_H2D
    const int env_streams = es_env ? atoi(es_env) : 2;
    const int nstreams = a.fmt == GIC_FMT_BC7 ? 1 : (env_streams < 1 ? 1 : (env_streams > 3 ? 3 : env_streams));
    const hipStream_t es[3] = {lane.enc, lane.enc2, lane.enc3};
    int rc = GIC_OK;
    size_t issued = 0;
    if (inline_up) e = hipEventRecord(lane.t_up0, lane.up);
    for (size_t k = 0; k < pieces.size() && !stop() && e == hipSuccess; ++k) {
        const Piece &p = pieces[k];
        if (inline_up) {
            e = hipMemcpyAsync(p.d_src, p.h_src, p.src_bytes, hipMemcpyHostToDevice, lane.up);
            if (e == hipSuccess) e = hipEventRecord(lane.ev_up[k], lane.up);
            if (e != hipSuccess) break;
        } else if (!uploaded.wait(k)) {
            break;
        }
        const hipStream_t s = es[k % nstreams];
        e = hipStreamWaitEvent(s, lane.ev_up[k], 0);
        if (e == hipSuccess && k == 0) e = hipEventRecord(lane.t_enc0, s);
        if (e != hipSuccess) break;
        rc = gic_hip_encode_rows_src(a.fmt, a.src_type, p.d_slice, a.width, a.height, 1, a.channels, a.row_pitch,
                                     p.y0, p.n, a.opt, p.h_out ? lane.zc + zc_off[k] : p.d_out, nullptr, s);
        if (rc != GIC_OK) break;
        e = hipEventRecord(lane.ev_enc[k], s);
        if (e != hipSuccess) break;
        issued = k + 1;
        encoded.post(issued);
    }
    // join: stream 0 waits for the other streams' last pieces
    for (int t = 1; t < nstreams && e == hipSuccess; ++t) {
        if ((size_t)t >= issued) break;
        const size_t last_t = issued - 1 - ((issued - 1 + nstreams - t) % nstreams);   // the last piece k with k % nstreams == t
        e = hipStreamWaitEvent(lane.enc, lane.ev_enc[last_t], 0);
    }
    if (inline_up && e == hipSuccess) e = hipEventRecord(lane.t_up1, lane.up);
    if (issued && e == hipSuccess) e = hipEventRecord(lane.t_enc1, lane.enc);
    encoded.fail();
    if (rc != GIC_OK || e != hipSuccess) halt.store(true);   // the uploader stops at its next piece
    uploader.join();
    downloader.join();
    populator.join();
    hipError_t ee = hipStreamSynchronize(lane.enc);
    if (e == hipSuccess) e = ee;
    ee = hipStreamSynchronize(lane.enc2);
    if (e == hipSuccess) e = ee;
    ee = hipStreamSynchronize(lane.enc3);
    if (e == hipSuccess) e = ee;
    const hipError_t eu = hipStreamSynchronize(lane.up);
    if (e_up == hipSuccess) e_up = eu;
    if (rc != GIC_OK) return rc;
    if (e != hipSuccess || e_up != hipSuccess || e_dn != hipSuccess) return GIC_EHIP;
    if (times && issued == pieces.size()) {
        times->h2d_ms = span_ms(lane.t_up0, lane.t_up1);
        times->encode_ms = span_ms(lane.t_enc0, lane.t_enc1);
        times->d2h_ms = d2h_span;
    }
    return GIC_OK;
}

}  // namespace gic
