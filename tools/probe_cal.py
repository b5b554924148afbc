"""Random-probe rate of the fingerprint-set access pattern (rmc_probe_bench)
over table sizes from L2/Infinity-Cache resident to far beyond: the ceiling a
partitioned (cache-resident) probe pass could reach versus the HBM-random one.

    python tools/probe_cal.py [--sizes-mb 64,256,...] [--accesses N] [--modes 0,1]

Prints one JSON line per (size, mode).  Run under `rocprofv3 --pmc FETCH_SIZE`
with a single size to calibrate FETCH_SIZE bytes per random 8-B probe.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))

import rmc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="16,64,128,256,512,2048,16384,65536")
    ap.add_argument("--accesses", type=int, default=1 << 31)
    ap.add_argument("--modes", default="0,1")
    a = ap.parse_args()
    for mb in [int(x) for x in a.sizes_mb.split(",")]:
        for mode in [int(x) for x in a.modes.split(",")]:
            r = rmc.probe_bench(device=0, table_bytes=mb << 20, accesses=a.accesses, mode=mode)
            print(json.dumps({"table_mb": mb, "mode": "load" if mode == 0 else "cas",
                              "accesses": a.accesses, "rate_per_s": r}), flush=True)


if __name__ == "__main__":
    main()
