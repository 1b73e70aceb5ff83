"""Per-launch HBM traffic of the env-step kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; they
cannot share a pass on gfx950), following /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so it is
doubled (the kernel's reads are narrower and uncalibrated, so the doubled figure is an upper estimate).

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv --arenas 4096 --precision fp32 [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import json
import statistics


def per_launch(path, counter):
    """median per launch of the step-kernel instantiation with the most traffic (the (2,4) bench also launches the
    wide rerun kernel after every step, nearly always over an empty list); returns (bytes, launches, kernel)"""
    by = {}
    for r in csv.DictReader(open(path)):
        if "step_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            by.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    if not by:
        raise SystemExit(f"no step_kernel {counter} rows in {path}")
    k = max(by, key=lambda n: statistics.median(by[n]))
    return statistics.median(by[k]) * 1024.0, len(by[k]), k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--arenas", type=int, default=4096)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    fetch, nf, kname = per_launch(a.fetch, "FETCH_SIZE")
    write, nw, _ = per_launch(a.write, "WRITE_SIZE")
    rec = {"kernel": kname, "arenas": a.arenas, "precision": a.precision, "A": a.arms, "K": a.objects,
           "fetch_size_bytes_raw": fetch, "write_size_bytes": write, "launches": [nf, nw],
           "hbm_bytes_per_launch": 2.0 * fetch + write,
           "note": "median over the launches of the kernel (pre-roll, warm-up and timed steps); FETCH_SIZE doubled per the "
                   "gfx950 guide (upper estimate for narrow reads); TCC -> memory-fabric bytes: the spilled per-arena "
                   "scratch blocks (contact records, Hessian) that leave the L2 count here whether the MALL or HBM "
                   "serves them"}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
