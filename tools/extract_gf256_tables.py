"""Extracts the numeric values of the reference's GF(2^8) tables into
tests/golden/gf256_tables.json (numbers only; the reference's file text is not
copied). Source: hadoop-common-project/hadoop-common/src/main/java/org/apache/
hadoop/io/erasurecode/rawcoder/util/GF256.java — GF_BASE (powers of the
primitive element, 0x11D) and GF_LOG_BASE (its log table, with log(1) stored
as 0xff), the literal tables behind RSRawEncoder / RSRawDecoder, the pure-Java
port of ISA-L's RS coder that the reference's interop tests
(TestRSRawCoderInteroperable1/2) hold equal to the native one behind the `nrs`
codec. tests/test_nrs_apache.py pins the oracle's and the engine's field
tables to these values.

Run in the build container (the reference does not exist on the GPU boxes):
    python tools/extract_gf256_tables.py [/root/reference]
"""
import json
import os
import re
import sys

REL = ("hadoop-common-project/hadoop-common/src/main/java/org/apache/hadoop/io/erasurecode/rawcoder/util/"
       "GF256.java")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def extract(text):
    out = {}
    for name in ("GF_BASE", "GF_LOG_BASE"):
        m = re.search(r"static\s+final\s+byte\[\]\s+" + name + r"\s*=\s*new\s+byte\[\]\s*\{(.*?)\};", text, re.S)
        if not m:
            raise ValueError(f"{name} not found")
        vals = [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]+)", m.group(1))]
        out[name] = {"line": text[:m.start()].count("\n") + 1, "values": vals}
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    with open(os.path.join(ref, REL)) as f:
        tabs = extract(f.read())
    out = {"_source": f"{REL} (reference @ /root/reference), numeric values of GF_BASE and GF_LOG_BASE; "
                      "extracted by tools/extract_gf256_tables.py"}
    for name, t in tabs.items():
        out[name] = {"reference_line": t["line"], "values": t["values"]}
    dst = os.path.join(ROOT, "tests", "golden", "gf256_tables.json")
    with open(dst, "w") as f:
        json.dump(out, f)
        f.write("\n")
    print("wrote", dst, {k: len(v["values"]) for k, v in tabs.items()})


if __name__ == "__main__":
    main()
