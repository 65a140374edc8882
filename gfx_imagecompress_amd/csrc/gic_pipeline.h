// gic_pipeline.h -- the host-image pipeline behind Image_Compress* and
// gic_encode_multi (internal; not part of the C ABI).
//
// The reference's image wrappers take a host image and return a host image
// (amd_bc1_compressor.cpp:36-70, amd_bc7_compressor.cpp:25-81).  On a GPU that
// means upload, encode, download; done in series the 8K BC1 call is bound by
// the 256 MiB upload, not by the 7 ms encode.  The pipeline cuts the block rows
// into pieces and runs three stages concurrently on one device ("lane"):
//   upload   (a helper thread, running ahead: piece k+1 crosses PCIe while
//             piece k encodes),
//   encode   (the calling thread, gic_hip_encode_rows_src on the lane's
//             encode streams, each piece waiting on its own upload event;
//             consecutive pieces alternate between two streams, so the tail of
//             one launch overlaps the next -- 16 pieces of an 8K BC1 image
//             then cost what one launch does, profiles/r06_pieces.txt),
//   download (a helper thread: the kernels write a host image's blocks straight
//             into pinned host memory; piece k is copied into the image while
//             k+1 encodes).
// Stages hand pieces over through per-piece events and counters; every event,
// stream and staging buffer belongs to the lane and is reused across calls.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

#include "../../include/gfx_imagecompress_amd/gic.h"

namespace gic {

// How a piece's source bytes reach the device (GIC_H2D: pageable | staged | register).
//   pageable: hipMemcpyAsync straight from the caller's (pageable) memory; the
//             runtime stages it through its own pinned buffers;
//   staged:   the upload thread copies each piece into a ring of pinned slots
//             and DMAs from there (the CPU copy of piece k+1 overlaps the DMA
//             of piece k);
//   register: the caller's range is page-locked in place (hipHostRegister)
//             for the call and DMAed directly.
enum class H2D : int { Pageable = 0, Staged = 1, Register = 2 };
H2D h2d_mode();

struct Piece {
    uint32_t slice, y0, n;     // block rows [y0, y0 + n) of one slice
    const uint8_t *h_src;      // the host source bytes the piece reads
    size_t src_bytes;
    uint8_t *d_src;            // where they land on the device
    const uint8_t *d_slice;    // the slice's pixel row 0 as the kernels address it
    uint8_t *d_out;            // the piece's packed blocks (device)
    uint8_t *h_out;            // host copy of them, or nullptr (blocks stay on the device)
    size_t out_bytes;
};

struct EncodeArgs {
    gic_format fmt;
    gic_source src_type;
    uint32_t width, height, channels;
    size_t row_pitch;
    const gic_options *opt;
};

// Per-device streams, events and pinned staging, reused across calls.
struct Lane {
    int device = -1;
    hipStream_t up = nullptr, enc = nullptr, enc2 = nullptr, enc3 = nullptr, down = nullptr;
    std::vector<hipEvent_t> ev_up, ev_enc;              // one per piece (grown on demand)
    hipEvent_t t_up0 = nullptr, t_up1 = nullptr, t_enc0 = nullptr, t_enc1 = nullptr;   // stage spans (timing)
    uint8_t *stage = nullptr;                            // pinned ring (H2D::Staged)
    size_t stage_slot = 0;
    uint8_t *zc = nullptr;                               // pinned outputs the kernels write (host images)
    size_t zc_cap = 0;
    bool zc_nc = false;                                  // allocated non-coherent (GIC_PIPE_ZC_NC)
    hipError_t init(int dev);
    hipError_t reserve_events(size_t pieces);
    hipError_t reserve_stage(size_t slot_bytes);
    hipError_t reserve_zc(size_t bytes, bool non_coherent = false);
    void release();
};

// Completed block rows, shared between the lanes' download stages and the
// thread that reports progress (the caller's).
struct Progress {
    std::mutex m;
    std::condition_variable cv;
    std::vector<uint64_t> done;   // rows completed per lane, in the lane's row order
    int finished = 0;             // lanes whose stages have all returned
    std::atomic<bool> abort{false};
    void add(int lane, uint64_t rows)
    {
        {
            std::lock_guard<std::mutex> lk(m);
            done[lane] += rows;
        }
        cv.notify_all();
    }
    void finish()
    {
        {
            std::lock_guard<std::mutex> lk(m);
            ++finished;
        }
        cv.notify_all();
    }
};

struct StageTimes {
    double h2d_ms = 0, encode_ms = 0;   // first start -> last end of each stage (HIP events)
    double d2h_ms = 0;                  // first -> last copy into the host image (host clock)
};

// Runs `pieces` (in order) through `lane` on the calling thread plus two helper
// threads.  `progress` (may be null) gets += piece.n for lane `lane_index`
// once a piece is complete (downloaded, or encoded when h_out is null); when
// progress->abort is set the stages stop between pieces.  Returns GIC_OK or a
// gic error code; `times` (may be null) gets the stage spans.
int run_pieces(Lane &lane, const EncodeArgs &a, const std::vector<Piece> &pieces, Progress *progress, int lane_index,
               StageTimes *times);

// Block rows per piece: `first` for the first piece of a range, `per` for
// the others.  The lane-per-block kernels take about 2^18 blocks a piece (their
// launches overlap on two streams, so small pieces cost nothing and the first
// upload is short); BC7 calls carry a multi-stage pipeline of their own and
// lose 5-15 % per extra call (profiles/r06_pieces.txt), so BC7 takes a small
// first piece (1/16 of the range: its upload is all the encode waits for) and
// the rest in one.  GIC_PIECE_BLOCKS overrides both with a block count (tests).
struct PiecePlan {
    uint32_t first, per;
};
PiecePlan piece_plan(gic_format fmt, uint32_t blocks_x, uint64_t rows);

// Cuts the slice-major block rows [first, first + rows) into pieces (plan)
// that do not cross slices.  Source bytes come from h_src (slices x height rows
// of pitch bytes) and land in d_src_slab packed in order; each piece's blocks
// go to d_out + (row - first) * row_bytes (and h_out likewise, if not null).
std::vector<Piece> make_pieces(uint64_t first, uint64_t rows, const PiecePlan &plan, uint32_t blocks_y,
                               uint32_t height, size_t pitch, size_t row_bytes, const uint8_t *h_src,
                               uint8_t *d_src_slab, uint8_t *d_out, uint8_t *h_out);
// the source bytes make_pieces lays out for that range
size_t slab_bytes(uint64_t first, uint64_t rows, uint32_t blocks_y, uint32_t height, size_t pitch);

// One device's share of a host-image call.
struct LaneJob {
    Lane *lane = nullptr;
    std::vector<Piece> pieces;
    uint64_t first_row = 0, rows = 0;   // the slice-major block rows it covers
    std::function<int()> after;         // run on the lane's thread after its pieces (a send), or empty
    StageTimes times;
    double wall_ms = 0;                 // its pieces plus `after`, host clock
    int rc = GIC_OK;
};

typedef bool (*ProgressFn)(void *user, float percentage);

// Runs every job on a thread of its own (a single job without a callback on
// the calling thread) and, when cb is set, reports progress from the calling
// thread exactly as the reference's loops do (amd_bc1_compressor.cpp:64-68):
// cb(user, 100 * (y * bx) / (bx * by)) for every block row y of every slice,
// slice-major, each once that row is complete on whichever device holds it.  A
// callback returning true stops every job between pieces and the call returns
// GIC_EABORT.  Otherwise returns GIC_OK or the first job's error.
int drive(std::vector<LaneJob> &jobs, const EncodeArgs &a, uint32_t blocks_x, uint32_t blocks_y, ProgressFn cb,
          void *user);

// A lane with its device buffers (source slab, packed blocks), reused across calls.
struct LaneBuffers {
    Lane lane;
    uint8_t *src = nullptr, *dst = nullptr;
    size_t src_cap = 0, dst_cap = 0;
    hipError_t reserve(size_t src_bytes, size_t dst_bytes);   // on lane.device
    void release();
};

// Host image in, host blocks out over one or more lanes: the slice-major block
// rows are split as gic_multi_split does, each lane pipelines its range (upload /
// encode / download straight into h_out at the range's offset -- no device
// gather, every device has its own PCIe link), progress as drive().  `rep`
// (may be null) gets the call's report.
int encode_host(const std::vector<LaneBuffers *> &lanes, const EncodeArgs &a, const uint8_t *h_src, uint32_t slices,
                uint8_t *h_out, ProgressFn cb, void *user, gic_host_report *rep);

// The same over the process-wide device-list group of gic_encode_multi
// (GIC_DEVICES for the Image_Compress* entry points).
int encode_host_devices(const std::vector<int> &devices, const EncodeArgs &a, const uint8_t *h_src, uint32_t slices,
                        uint8_t *h_out, ProgressFn cb, void *user, gic_host_report *rep);

double now_ms();   // host steady clock

// Data of a host image this library creates (Image_CreateNoClear; released with
// free()): large images are 2 MiB aligned and advised for transparent huge
// pages, so the copy-out stage does not spend its time in 4 KiB page faults
// (a fresh 32 MiB malloc is 8192 first-touch faults, several ms on one thread).
void *alloc_image_data(size_t bytes);

}  // namespace gic
