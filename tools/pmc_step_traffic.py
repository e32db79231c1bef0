"""Summarise tools/pmc_step_traffic.sh: per-launch HBM bytes of each timed step kernel.

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of 16-byte-per-lane reads (MI355X_MICROARCH.md, HBM), which both step-kernel forms use
(buffer_load_dwordx4, and buffer_load ... lds), so it is doubled; WRITE_SIZE is exact for 16-byte stores.
Infinity-Cache hits count as fetches.  Median over the dispatches of the layer's kernel.
"""
import csv
import glob
import json
import os
import sys

NAMES = ["enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2"]


def per_dispatch(path, counter):
    vals = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "uconv_kernel" in k and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sorted(vals)[len(vals) // 2] if vals else None


def main():
    out, layers = sys.argv[1], sys.argv[2:]
    res = {"per_launch_bytes": {}, "detail": {},
           "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over tools/step_times.py "
                     f"--layers L --dtype {os.environ.get('DTYPE', 'fp32')} (the instance the loop runs), B=8 16x64 "
                     "latent, median dispatch; FETCH_SIZE x2 (gfx950)"}
    for L in layers:
        name = NAMES[int(L)]
        fetch_kib = per_dispatch(os.path.join(out, f"l{L}_FETCH_SIZE"), "FETCH_SIZE")
        write_kib = per_dispatch(os.path.join(out, f"l{L}_WRITE_SIZE"), "WRITE_SIZE")
        if fetch_kib is None or write_kib is None:
            continue
        read_b = 2.0 * fetch_kib * 1024.0
        write_b = write_kib * 1024.0
        res["per_launch_bytes"][name] = read_b + write_b
        res["detail"][name] = {"fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
                               "read_bytes_corrected": read_b, "write_bytes": write_b}
    with open(os.path.join(out, "pmc_traffic_step.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
