"""Extract the message/field table of the reference's checkpoint protos into
tests/golden/proto_fields.json (data only), so the storage tests can pin this build's
programmatic descriptors to the reference wire format without reading the reference at
test time.

    python tests/golden/make_proto_fields.py /root/reference/src/spectralmc/proto
"""

from __future__ import annotations

import json
import os
import re
import sys

FIELD = re.compile(r"^\s*(repeated\s+)?(map<\s*\w+\s*,\s*\w+\s*>|[\w.]+)\s+(\w+)\s*=\s*(\d+)\s*;")


def parse(path: str) -> dict[str, list[list]]:
    out: dict[str, list[list]] = {}
    msg = None
    depth = 0
    for raw in open(path):
        line = raw.split("//")[0]
        m = re.match(r"^\s*message\s+(\w+)\s*\{", line)
        if m and depth == 0:
            msg, depth = m.group(1), 1
            out[msg] = []
            continue
        if msg is None:
            continue
        f = FIELD.match(line)
        if f and depth == 1:
            kind = re.sub(r"\s+", "", f.group(2))
            out[msg].append([f.group(3), int(f.group(4)), kind, bool(f.group(1))])
        depth += line.count("{") - line.count("}")
        if depth == 0:
            msg = None
    return out


def main() -> None:
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/spectralmc/proto"
    table = {}
    for name in ("common.proto", "tensors.proto"):
        table.update(parse(os.path.join(src, name)))
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "proto_fields.json")
    with open(dst, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(f"wrote {dst}: {sorted(table)}")


if __name__ == "__main__":
    main()
