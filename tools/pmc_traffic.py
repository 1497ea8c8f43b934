"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) into per-launch HBM traffic of k_batch.

Counters and corrections (MI355X_MICROARCH.md §HBM):
  FETCH_SIZE, WRITE_SIZE are in KiB and count the L2's memory-side (fabric) requests, Infinity-Cache
  hits included.  On gfx950 FETCH_SIZE reports half of the bytes of wide coalesced reads, so the
  corrected read bytes are 2 x FETCH_SIZE x 1024; WRITE_SIZE is taken as is.
The first k_batch dispatch of each bench run is the parity-gate pass (it also copies every frame
out), so it is dropped; the remaining dispatches are the timed-path launches.
Prints one JSON object: per-launch read/write bytes (median over launches), L2 hit rate.
"""
import csv
import glob
import json
import os
import statistics
import sys


KERNEL = "k_batch"


def per_dispatch(d):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            kn = row["Kernel_Name"]
            if KERNEL == "h265" and "k_h265_" not in kn:
                continue
            if KERNEL != "h265" and not kn.startswith(KERNEL):
                continue
            key = int(row["Dispatch_Id"])
            vals.setdefault(key, {})
            name = row["Counter_Name"]
            vals[key][name] = vals[key].get(name, 0.0) + float(row["Counter_Value"])
            for g in ("Grid_Size", "Grid_Size_X"):
                if g in row and row[g]:
                    vals[key]["_grid"] = float(row[g])
            vals[key]["_name"] = kn
    keys = sorted(vals)[1:] if KERNEL == "k_batch" else sorted(vals)  # k_batch: drop the parity-gate launch
    return [vals[k] for k in keys]


def h265(root, label, out):
    """The H.265 legs: every k_h265_* dispatch of the run (2 passes of the 8-picture stream + its warmup),
    summed, per picture (one k_h265_ctu_index per picture with blocks)."""
    out["preset"] = "c_h265_1080p_pb_s1" if label == "h265_pb" else "c_h265_1080p_s1"
    out["frames"] = 8
    fetch = per_dispatch(os.path.join(root, "FETCH_SIZE"))
    write = per_dispatch(os.path.join(root, "WRITE_SIZE"))
    pics_f = max(1, sum(1 for v in fetch if "k_h265_ctu_index" in v["_name"]))
    pics_w = max(1, sum(1 for v in write if "k_h265_ctu_index" in v["_name"]))
    f = sum(v["FETCH_SIZE"] for v in fetch) / pics_f
    w = sum(v["WRITE_SIZE"] for v in write) / pics_w
    out["pictures"] = pics_f
    out["fetch_size_kib_per_picture"] = round(f, 1)
    out["write_size_kib_per_picture"] = round(w, 1)
    out["read_bytes_raw"] = int(f * 1024)
    out["read_bytes_doubled"] = int(2 * f * 1024)
    out["write_bytes"] = int(w * 1024)
    by = {}
    for v in fetch:
        k = v["_name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        by[k] = by.get(k, 0.0) + v["FETCH_SIZE"] * 1024 / pics_f
    out["read_bytes_raw_by_kernel"] = {k: int(x) for k, x in sorted(by.items())}
    bw = {}
    for v in write:
        k = v["_name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        bw[k] = bw.get(k, 0.0) + v["WRITE_SIZE"] * 1024 / pics_w
    out["write_bytes_by_kernel"] = {k: int(x) for k, x in sorted(bw.items())}
    # FETCH_SIZE x 2 holds for wide coalesced streaming reads (MI355X_MICROARCH.md §HBM); the deblocking and
    # SAO passes are such reads, the CTU kernel's sample / record reads narrower: both bounds reported,
    # the doubled figure (the upper bound) as the traffic
    out["traffic_bytes_per_picture"] = out["read_bytes_doubled"] + out["write_bytes"]
    out["traffic_bytes_per_picture_raw"] = out["read_bytes_raw"] + out["write_bytes"]
    # the CTU kernels' wave states and instruction mix (SQ groups, when collected): sums over their dispatches, per
    # picture; the wave-cycle counters are quad-cycles (MI355X_MICROARCH.md §PMC: WAIT_ANY + WAIT_INST_ANY +
    # ACTIVE_INST_ANY ~ WAVE_CYCLES)
    sq = {}
    for d in sorted(glob.glob(os.path.join(root, "SQ_*"))):
        for v in per_dispatch(d):
            if "k_h265_ctu_" not in v["_name"]:
                continue
            for k, x in v.items():
                if k.startswith("SQ_") or k.startswith("GRBM_"):
                    sq[k] = sq.get(k, 0.0) + x
    if sq:
        n = max(1, pics_f)
        out["ctu_kernel_counters_per_picture"] = {k: round(x / n, 1) for k, x in sorted(sq.items())}
        wc = sq.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            out["ctu_kernel_wave_state_fractions"] = {k: round(sq.get(k, 0.0) / wc, 4) for k in (
                "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                "SQ_WAIT_INST_LDS")}


def main():
    global KERNEL
    root = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else "k_batch"
    KERNEL = {"k_batch8": "k_batch", "h265_pb": "h265"}.get(label, label)
    out = {"kernel": KERNEL, "source": "rocprofv3 --pmc, one pass per counter group (tools/gpu_pmc.sh)"}
    if label == "k_batch8":
        out["preset"] = "c3x8"  # bench.py gpu_recon_streams: the 8 C4 streams in one replay
    if KERNEL == "h265":
        h265(root, label, out)
        print(json.dumps(out, indent=1))
        return
    fetch = per_dispatch(os.path.join(root, "FETCH_SIZE"))
    write = per_dispatch(os.path.join(root, "WRITE_SIZE"))
    hit = per_dispatch(os.path.join(root, "TCC_HIT_sum_TCC_MISS_sum"))
    if fetch:
        f = statistics.median(v["FETCH_SIZE"] for v in fetch)
        out["fetch_size_kib"] = f
        out["read_bytes"] = int(2 * f * 1024)
        out["read_bytes_raw"] = int(f * 1024)  # FETCH_SIZE undoubled: the lower bound (narrow gathers)
        out["launches_read"] = len(fetch)
    if write:
        w = statistics.median(v["WRITE_SIZE"] for v in write)
        out["write_size_kib"] = w
        out["write_bytes"] = int(w * 1024)
    if "read_bytes" in out and "write_bytes" in out:
        out["traffic_bytes"] = out["read_bytes"] + out["write_bytes"]
        out["traffic_bytes_raw"] = out["read_bytes_raw"] + out["write_bytes"]
    if KERNEL == "k_picture" and fetch and write and all("_grid" in v for v in fetch + write):
        # the decode path launches 1..4 pictures at once: bytes per picture (sum over launches / pictures),
        # which bench.py scales by its own pictures per launch.  A 1080p picture is 34 row-pair workgroups of
        # 256 lanes without inter MBs, else 80 inter workers + 12 row workgroups (runtime.hip
        # picture_blocks_dp): a launch's grid names its picture counts uniquely
        def pics_of(grid):
            g = int(round(grid / 256))
            for n in range(1, 5):
                for i in range(n + 1):
                    if 34 * i + 92 * (n - i) == g:
                        return n
            return g / 92.0
        pics_f = sum(pics_of(v["_grid"]) for v in fetch)
        pics_w = sum(pics_of(v["_grid"]) for v in write)
        out["traffic_bytes_per_picture"] = int(2 * 1024 * sum(v["FETCH_SIZE"] for v in fetch) / max(1.0, pics_f) +
                                              1024 * sum(v["WRITE_SIZE"] for v in write) / max(1.0, pics_w))
        out["traffic_bytes_per_picture_raw"] = int(1024 * sum(v["FETCH_SIZE"] for v in fetch) / max(1.0, pics_f) +
                                                  1024 * sum(v["WRITE_SIZE"] for v in write) / max(1.0, pics_w))
        out["pictures_per_launch"] = round(pics_f / len(fetch), 3)
    if hit:
        h = statistics.median(v["TCC_HIT_sum"] for v in hit)
        m = statistics.median(v["TCC_MISS_sum"] for v in hit)
        out["l2_hit_rate"] = round(h / max(1.0, h + m), 4)
    sq = per_dispatch(os.path.join(root, "SQ_WAVES_SQ_WAVE_CYCLES_SQ_WAIT_ANY_SQ_WAIT_INST_ANY_SQ_ACTIVE_INST_ANY_"
                                         "SQ_ACTIVE_INST_VALU_SQ_INSTS_VALU_SQ_BUSY_CYCLES_GRBM_GUI_ACTIVE"))
    if sq:
        med = {k: statistics.median(v.get(k, 0.0) for v in sq) for k in sq[0] if not k.startswith("_")}
        wc = max(1.0, med.get("SQ_WAVE_CYCLES", 0.0))
        out["sq"] = {k: int(v) for k, v in sorted(med.items())}
        # fractions of wave-resident time (quad-cycles): parked on waitcnt / barrier, stalled at issue,
        # issuing any instruction, issuing VALU
        out["sq_frac"] = {"wait_any": round(med.get("SQ_WAIT_ANY", 0) / wc, 4),
                          "wait_inst_any": round(med.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
                          "active_inst_any": round(med.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
                          "active_inst_valu": round(med.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
