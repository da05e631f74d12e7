"""Extracts the numeric values of the reference's CRC-32 slicing tables into
tests/golden/crc32_tables.json (numbers only; the reference's file text is not
copied). Source: hadoop-common-project/hadoop-common/src/main/native/src/org/
apache/hadoop/util/crc32_zlib_polynomial_tables.h — CRC32_T8_0 .. CRC32_T8_7,
the zlib-polynomial (0xEDB88320) slicing-by-8 tables libhadoop's native
checksums use; T8_0 is the byte table of java.util.zip.CRC32 and T8_j advances
a byte followed by j zero bytes. The engine's CRC kernels use T8_0..T8_3
(slicing by 4) and zero-append operators Z_n (lambdafs_amd/csrc/crc32.hpp);
tests/test_crc_tables.py pins both to these values.

Run in the build container (the reference does not exist on the GPU boxes):
    python tools/extract_crc_tables.py [/root/reference]
"""
import json
import os
import re
import sys

REL = ("hadoop-common-project/hadoop-common/src/main/native/src/org/apache/hadoop/util/"
       "crc32_zlib_polynomial_tables.h")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def extract(text):
    tables = {}
    for m in re.finditer(r"const\s+uint32_t\s+(CRC32_T8_[0-7])\s*\[\s*\]\s*=\s*\{(.*?)\};", text, re.S):
        vals = [int(x, 16) for x in re.findall(r"0x[0-9A-Fa-f]+", m.group(2))]
        if len(vals) != 256:
            raise ValueError(f"{m.group(1)}: {len(vals)} entries")
        line = text[:m.start()].count("\n") + 1
        tables[m.group(1)] = {"line": line, "values": vals}
    if sorted(tables) != [f"CRC32_T8_{j}" for j in range(8)]:
        raise ValueError(f"found {sorted(tables)}")
    return tables


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    path = os.path.join(ref, REL)
    with open(path) as f:
        tables = extract(f.read())
    out = {"_source": f"{REL} (reference @ /root/reference), numeric values of CRC32_T8_0..7; "
                      "extracted by tools/extract_crc_tables.py",
           "poly_reflected": "0xEDB88320"}
    for name in sorted(tables):
        out[name] = {"reference_line": tables[name]["line"], "values": tables[name]["values"]}
    dst = os.path.join(ROOT, "tests", "golden", "crc32_tables.json")
    with open(dst, "w") as f:
        json.dump(out, f)
        f.write("\n")
    print("wrote", dst)


if __name__ == "__main__":
    main()
