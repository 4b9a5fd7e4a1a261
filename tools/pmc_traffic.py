"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced read -> x2.  WRITE_SIZE is exact for 16-B and 4-B-per-lane streaming stores.
python tools/pmc_traffic.py <pmc_dir_fetch> <pmc_dir_write> <kernel-substring> [out.json]"""
import csv
import json
import statistics
import sys


def per_dispatch(path, counter, kname):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kname in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fdir, wdir, kname = sys.argv[1:4]
    f = per_dispatch(fdir + "/run_counter_collection.csv", "FETCH_SIZE", kname)
    w = per_dispatch(wdir + "/run_counter_collection.csv", "WRITE_SIZE", kname)
    fetch = statistics.median(f) * 1024 * 2
    write = statistics.median(w) * 1024
    out = {"kernel": kname, "dispatches": [len(f), len(w)], "fetch_bytes_corrected": fetch,
           "write_bytes": write, "traffic_bytes_per_launch": fetch + write,
           "note": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE as reported; KB->B x1024"}
    print(json.dumps(out))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
