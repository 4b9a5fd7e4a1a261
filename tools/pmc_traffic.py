"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB),
calibrated on known byte counts of the same access width (tools/pmc_calib.py: 4-B-per-lane
coalesced loads / stores, 512 MiB read and 256 MiB written, beyond the 256 MiB MALL).

MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads and
other widths are uncalibrated -> the factor is measured here instead of assumed.
python tools/pmc_traffic.py <fetch_dir> <write_dir> <calib_fetch_dir> <calib_write_dir> <kernel> [out.json]"""
import csv
import json
import statistics
import sys


def per_dispatch(path, counter, kname):
    vals = []
    for r in csv.DictReader(open(path + "/run_counter_collection.csv")):
        if r["Counter_Name"] == counter and kname in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    fdir, wdir, cfdir, cwdir, kname = sys.argv[1:6]
    n = 64 * 1024 * 1024
    cf = statistics.median(per_dispatch(cfdir, "FETCH_SIZE", "k_l1_partial"))
    cw = statistics.median(per_dispatch(cwdir, "WRITE_SIZE", "k_l1_backward"))
    f_fetch = (2 * n * 4) / cf
    f_write = (n * 4) / cw
    f = per_dispatch(fdir, "FETCH_SIZE", kname)
    w = per_dispatch(wdir, "WRITE_SIZE", kname)
    fetch = statistics.median(f) * f_fetch
    write = statistics.median(w) * f_write
    out = {"kernel": kname.rstrip(",") + ">", "dispatches": [len(f), len(w)], "fetch_factor": round(f_fetch, 4),
           "write_factor": round(f_write, 4), "fetch_bytes": fetch, "write_bytes": write,
           "traffic_bytes_per_launch": fetch + write,
           "note": "median per dispatch; FETCH_SIZE/WRITE_SIZE (KB) x calibration factor measured on "
                   "4-B-per-lane streaming kernels with known byte counts (tools/pmc_calib.py)"}
    print(json.dumps(out))
    if len(sys.argv) > 6:
        json.dump(out, open(sys.argv[6], "w"), indent=1)


if __name__ == "__main__":
    main()
