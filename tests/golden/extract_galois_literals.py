"""Extract the literal LOG_TABLE / EXP_TABLE values of the reference's
Galois.java (lines 58-92 and 102-169) into galois_tables.json.

Run once in the build container (it reads /root/reference, which does not exist
on the GPU box); the committed JSON holds only the table VALUES (data), which
pin the oracle's generated tables.  The Java `byte` literals are signed; they
are stored as unsigned 0..255.
"""
import json
import os
import re
import sys

SRC = "/root/reference/src/main/java/edu/cmu/reedsolomon/Galois.java"
HERE = os.path.dirname(os.path.abspath(__file__))


def table(text: str, name: str):
    m = re.search(name + r"\s*=\s*new\s+\w+\s*\[\]\s*\{(.*?)\};", text, re.S)
    if not m:
        sys.exit(f"{name} not found")
    return [int(v) for v in re.findall(r"-?\d+", m.group(1))]


def main():
    text = open(SRC).read()
    log = table(text, "LOG_TABLE")
    exp = [v & 0xFF for v in table(text, "EXP_TABLE")]
    assert len(log) == 256 and len(exp) == 510, (len(log), len(exp))
    out = {
        "source": "Galois.java:58-92 (LOG_TABLE), Galois.java:102-169 (EXP_TABLE); EXP bytes as unsigned",
        "log_table": log,
        "exp_table": exp,
    }
    with open(os.path.join(HERE, "galois_tables.json"), "w") as f:
        json.dump(out, f)
    print("wrote galois_tables.json", len(log), len(exp))


if __name__ == "__main__":
    main()
