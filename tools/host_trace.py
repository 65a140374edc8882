"""Timeline of the last host-image call in a rocprofv3 --kernel-trace
--memory-copy-trace csv directory (tools/time_host.py under the profiler):
uploads and encode kernels relative to the call's first upload.

    python tools/host_trace.py <dir> [--kernel bc1_image_kernel] [--pieces 16]
"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="bc1_image_kernel")
    ap.add_argument("--pieces", type=int, default=16)
    a = ap.parse_args()
    ks = [r for f in glob.glob(a.dir + "/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
    cs = [r for f in glob.glob(a.dir + "/**/*memory_copy_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:40], r["Stream_Id"]) for r in ks]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r["Direction"].replace("MEMORY_COPY_", ""),
            r["Stream_Id"]) for r in cs]
    ev.sort()
    enc = [e for e in ev if e[2] == "K" and a.kernel in e[3]]
    last = enc[-a.pieces:]
    t_first_k = last[0][0]
    ups = [e for e in ev if e[2] == "C" and e[3] == "HOST_TO_DEVICE" and e[0] <= last[-1][0]]
    # the call's uploads: the last `pieces` host-to-device copies before its last kernel started
    ups = ups[-a.pieces:]
    t0 = min(ups[0][0], t_first_k)
    window = [e for e in ev if e[0] >= t0 and e[0] <= last[-1][1]]
    print("start_ms   end_ms  dur_ms  kind  name  stream")
    for s, e, k, n, st in window:
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  {k} {n} {st}")
    kd = [(e - s) / 1e6 for s, e, *_ in last]
    print(f"encode kernels: {len(last)}, mean duration {sum(kd) / len(kd):.3f} ms, first start {(last[0][0] - t0) / 1e6:.3f} ms, "
          f"last end {(last[-1][1] - t0) / 1e6:.3f} ms; uploads end {(ups[-1][1] - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
