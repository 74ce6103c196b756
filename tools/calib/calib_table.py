"""FETCH_SIZE / WRITE_SIZE calibration table from two rocprofv3 --pmc passes over
tools/calib/calib_fetch (each kernel streams exactly 1 GiB once).

    python tools/calib/calib_table.py <fetch_dir> <write_dir> > profiles/<tag>_fetch_calibration.json

ratio = counter bytes (KB x 1024) / true bytes; the correction a kernel's counter needs is
1 / ratio for its dominant access width."""
import csv
import glob
import json
import os
import re
import sys

TRUE_BYTES = 1 << 30


def load(d, counter):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                m = re.search(r"\b(rd|wr)<(.*)>\s*\(", name)
                if not m:
                    continue
                key = f"{m.group(1)}<{m.group(2).strip()}>"
                vals.setdefault(key, []).append(float(row["Counter_Value"]) * 1024.0)
    return vals


def main(fetch_dir, write_dir):
    f = load(fetch_dir, "FETCH_SIZE")
    w = load(write_dir, "WRITE_SIZE")
    width = {"unsigned char": 1, "unsigned short": 2, "unsigned int": 4, "unsigned long": 8, "uint4": 16,
             "HIP_vector_type<unsigned int, 4u>": 16, "HIP_vector_type<unsigned int, 4u> ": 16}
    out = {"true_bytes_per_launch": TRUE_BYTES, "read": {}, "write": {}}
    for key, v in sorted(f.items()):
        if key.startswith("rd"):
            t = key[3:-1]
            out["read"][str(width.get(t, t))] = {"kernel": key, "fetch_size_bytes": min(v),
                                                 "ratio": round(min(v) / TRUE_BYTES, 4), "launches": len(v)}
    for key, v in sorted(w.items()):
        if key.startswith("wr"):
            t = key[3:-1]
            out["write"][str(width.get(t, t))] = {"kernel": key, "write_size_bytes": min(v),
                                                  "ratio": round(min(v) / TRUE_BYTES, 4), "launches": len(v)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
