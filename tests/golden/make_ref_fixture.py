"""Regenerate tests/golden/ref_tables.json from the reference's own compiled sources.

Builds oracle/_ref/ref_harness (oracle/Makefile target `ref`, compiled from /root/reference,
never shipped) and stores its JSON output as a committed fixture. Run here only: the GPU box
has no /root/reference.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    if not os.path.isdir("/root/reference"):
        print("reference not present; fixture left untouched")
        return 0
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_harness")], check=True,
                         capture_output=True, text=True).stdout
    data = json.loads(out)
    dst = os.path.join(ROOT, "tests", "golden", "ref_tables.json")
    with open(dst, "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print("wrote", dst)
    return 0


if __name__ == "__main__":
    sys.exit(main())
