"""Summarise tools/pmc_traffic.sh passes: per-launch HBM read / write bytes of each UNet conv layer.

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch; on gfx950 FETCH_SIZE reports
half the bytes of 16-byte-per-lane coalesced reads (MI355X_MICROARCH.md, HBM), so it is doubled here;
WRITE_SIZE is exact for 16-byte stores and float stores.  Infinity-Cache hits are counted as fetches.
"""
import csv
import glob
import json
import os
import sys

NAMES = ["enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1",
         "ca2.q", "ca2.kv", "ca2.out", "ca1.q", "ca1.kv", "ca1.out"]


def per_dispatch(path, counter):
    vals = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv_mfma" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sorted(vals)[len(vals) // 2] if vals else None


def main():
    out, layers = sys.argv[1], sys.argv[2:]
    res = {"per_launch_bytes": {}, "detail": {}, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_sum, "
                                                           "tools/prof_layer.py B=8 16x64 latent, median dispatch"}
    for L in layers:
        name = NAMES[int(L)]
        fetch_kib = per_dispatch(os.path.join(out, f"l{L}_FETCH_SIZE"), "FETCH_SIZE")
        write_kib = per_dispatch(os.path.join(out, f"l{L}_WRITE_SIZE"), "WRITE_SIZE")
        rdreq = per_dispatch(os.path.join(out, f"l{L}_TCC_EA0_RDREQ_sum"), "TCC_EA0_RDREQ_sum")
        if fetch_kib is None or write_kib is None:
            continue
        read_b = 2.0 * fetch_kib * 1024.0          # gfx950 FETCH_SIZE correction (x2)
        write_b = write_kib * 1024.0
        res["per_launch_bytes"][name] = read_b + write_b
        res["detail"][name] = {"fetch_size_kib": fetch_kib, "write_size_kib": write_kib, "tcc_ea0_rdreq": rdreq,
                               "read_bytes_corrected": read_b, "write_bytes": write_b}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
