#!/usr/bin/env python3
"""Transcribe the v1beta2 TopologyAssignment encoding vectors of the
reference's own table tests into a JSON fixture (text parse of the Go
composite literals; nothing of the reference is executed).

Source: /root/reference/pkg/util/tas/tas_assignment_test.go
  bothWaysTestCases  (:40-421)  internal <-> v1beta2 (V1Beta2From and InternalFrom)
  oneWayTestCases    (:424-...) v1beta2 -> internal only (InternalFrom)

    python tools/extract_encoding_goldens.py > tests/golden/tas_v1beta2_encoding.json
"""
from __future__ import annotations

import json
import re
import sys

SRC = "/root/reference/pkg/util/tas/tas_assignment_test.go"
TOKEN = re.compile(r'\s+|//[^\n]*|"(?:[^"\\]|\\.)*"|\[\]|[A-Za-z_][A-Za-z0-9_.]*|-?\d+|[&{}():,]')


def tokenize(text, base_line):
    toks = []
    line = base_line
    pos = 0
    while pos < len(text):
        m = TOKEN.match(text, pos)
        if not m:
            raise ValueError(f"unexpected {text[pos:pos + 20]!r} at line {line}")
        t = m.group(0)
        if not (t.isspace() or t.startswith("//")):
            toks.append((t, line))
        line += t.count("\n")
        pos = m.end()
    return toks


class Parser:
    def __init__(self, toks):
        self.toks = toks
        self.i = 0

    def peek(self, k=0):
        return self.toks[self.i + k][0] if self.i + k < len(self.toks) else None

    def take(self, want=None):
        t, line = self.toks[self.i]
        if want is not None and t != want:
            raise ValueError(f"expected {want!r}, got {t!r} at line {line}")
        self.i += 1
        return t

    def value(self):
        t = self.peek()
        if t == "&":
            self.take()
            return self.value()
        if t == "new" or t == "int32":
            self.take()
            self.take("(")
            v = self.value()
            self.take(")")
            return v
        if t.startswith('"'):
            self.take()
            return json.loads(t)
        if re.fullmatch(r"-?\d+", t):
            self.take()
            return int(t)
        if t == "[]":  # []T{...}
            self.take()
            self.take()  # element type
            return self.composite()
        if t == "{":
            return self.composite()
        if t in ("nil", "true", "false"):
            self.take()
            return {"nil": None, "true": True, "false": False}[t]
        self.take()  # type name
        return self.composite()

    def composite(self):
        line = self.toks[self.i][1]
        self.take("{")
        keyed, items = {}, []
        while self.peek() != "}":
            if self.peek(1) == ":" and re.fullmatch(r"[A-Za-z_]\w*", self.peek()):
                k = self.take()
                self.take(":")
                keyed[k] = self.value()
            else:
                items.append(self.value())
            if self.peek() == ",":
                self.take()
        self.take("}")
        if keyed:
            keyed["_line"] = line
            return keyed
        return items


def extract(src, var):
    m = re.search(r"var %s = \[\]testCase" % var, src)
    start = src.index("{", m.end())
    depth, j = 0, start
    while True:
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    line = src.count("\n", 0, start) + 1
    return Parser(tokenize(src[start:j + 1], line)).composite()


def internal(d):
    if d is None:
        return None
    return {"levels": d.get("Levels", []),
            "domains": [{"values": x["Values"], "count": x["Count"]} for x in d.get("Domains", [])]}


def v1beta2(d):
    if d is None:
        return None
    slices = []
    for s in d.get("Slices", []):
        pc = s.get("PodCounts", {})
        vpl = []
        for v in s.get("ValuesPerLevel", []):
            if "Universal" in v:
                vpl.append({"universal": v["Universal"]})
            else:
                ind = v["Individual"]
                e = {"roots": ind.get("Roots", [])}
                if "Prefix" in ind:
                    e["prefix"] = ind["Prefix"]
                if "Suffix" in ind:
                    e["suffix"] = ind["Suffix"]
                vpl.append({"individual": e})
        slices.append({"domainCount": s["DomainCount"],
                       "podCounts": {"universal": pc["Universal"]} if "Universal" in pc
                       else {"individual": pc.get("Individual", [])},
                       "valuesPerLevel": vpl})
    return {"levels": d.get("Levels", []), "slices": slices}


def main():
    src = open(SRC).read()
    cases = []
    for var, both in (("bothWaysTestCases", True), ("oneWayTestCases", False)):
        for c in extract(src, var):
            cases.append({"name": c["name"], "line": c["_line"], "bothWays": both,
                          "internal": internal(c.get("internal")), "v1beta2": v1beta2(c.get("v1beta2")),
                          "podCounts": c.get("podCounts", []), "totalDomainCount": c.get("totalDomainCount", 0)})
    json.dump({"source": "pkg/util/tas/tas_assignment_test.go", "cases": cases}, sys.stdout, indent=1)
    sys.stdout.write("\n")


if __name__ == "__main__":
    main()
