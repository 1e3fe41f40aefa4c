#!/usr/bin/env python3
"""Golden-vector extractor for the TAS evaluation path.

Reads Kueue's own table test ``pkg/cache/scheduler/tas_cache_test.go``
(``TestFindTopologyAssignments``, reference :55-6341) **as text**, evaluates the
subset of Go expression syntax the table uses (composite literals, the
``testingnode``/``testingpod`` builder chains, ``resource.MustParse``,
``ptr.To``/``new``), and writes one JSON fixture per case to
``tests/golden/tas_find_topology_assignments.json``.

Nothing from the reference is executed, imported or copied: the output is data
(inputs + the expected outputs written in the reference test).  The fixture is
committed; this script is only needed to regenerate it, and only where
``/root/reference`` exists.

Fixture schema (one entry per case)::

  {"name": str, "line": int, "scope": "in" | "out:<reason>",
   "featureGates": {gate: bool},
   "levels": [str], "nodeLabels": {k: v},
   "nodes": [{"name", "labels", "allocatable": {res: int}, "taints": [..],
              "unschedulable": bool, "conditions": [{"type","status"}]}],
   "pods":  [{"name", "namespace", "nodeName", "phase", "requests": {res: int}}],
   "podSets": [{"name", "topologyRequest": {...}|null, "requests": {res:int},
                "count", "tolerations": [...], "nodeSelector": {..}|null,
                "podSetGroupName": str|null,
                "wantAssignment": {"levels", "domains": [{"values","count"}]}|null,
                "wantReason": str}]}

Resource quantities are converted exactly as ``resources.ResourceValue``
(reference pkg/resources/requests.go:106-111): cpu -> milli-units (ceil),
everything else -> integer units (ceil).
"""
from __future__ import annotations

import json
import math
import os
import re
import sys
from fractions import Fraction

REF_TEST = "pkg/cache/scheduler/tas_cache_test.go"

# ----------------------------------------------------------------------------
# Tokenizer (Go subset)
# ----------------------------------------------------------------------------
_TOKEN_RE = re.compile(
    r"""
    (?P<ws>[ \t\r\n]+)
  | (?P<lcomment>//[^\n]*)
  | (?P<bcomment>/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:\\.|[^"\\])*")
  | (?P<num>\d+(?:\.\d+)?)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>:=|\.\.\.|&&|\|\||==|!=|<=|>=|\+\+|--|[{}()\[\],:;.*&=+\-<>!/%|])
    """,
    re.VERBOSE | re.DOTALL,
)


class Tok:
    __slots__ = ("kind", "val", "line")

    def __init__(self, kind, val, line):
        self.kind, self.val, self.line = kind, val, line

    def __repr__(self):
        return f"Tok({self.kind},{self.val!r},L{self.line})"


def tokenize(src: str):
    toks = []
    pos, line = 0, 1
    while pos < len(src):
        m = _TOKEN_RE.match(src, pos)
        if not m:
            raise SyntaxError(f"cannot tokenize at line {line}: {src[pos:pos + 40]!r}")
        kind = m.lastgroup
        val = m.group(kind)
        if kind not in ("ws", "lcomment", "bcomment"):
            if kind == "str":
                val = json.loads(val)  # Go interpreted strings used here are JSON-compatible
            elif kind == "raw":
                kind, val = "str", val[1:-1]
            toks.append(Tok(kind, val, line))
        line += val.count("\n") if kind in ("ws", "bcomment") else 0
        pos = m.end()
    return toks


# ----------------------------------------------------------------------------
# AST (tiny)
# ----------------------------------------------------------------------------
class Lit:  # string / number
    def __init__(self, v):
        self.v = v


class Name:  # possibly qualified: "corev1.ResourceCPU"
    def __init__(self, n, line):
        self.n, self.line = n, line


class Call:
    def __init__(self, fn, args, line):
        self.fn, self.args, self.line = fn, args, line


class Method:
    def __init__(self, recv, name, args, line):
        self.recv, self.name, self.args, self.line = recv, name, args, line


class Composite:
    def __init__(self, typ, elems, line):
        self.typ, self.elems, self.line = typ, elems, line  # elems: list of (key|None, value)


class Unary:
    def __init__(self, op, x):
        self.op, self.x = op, x


class Closure:
    def __init__(self, line):
        self.line = line


GO_PACKAGES = {"testingnode", "testingpod", "resource", "ptr", "corev1", "kueue", "tas",
               "resources", "features", "fmt", "utiltestingapi", "featuregate", "utiltas"}


class Parser:
    def __init__(self, toks, i=0):
        self.t, self.i = toks, i

    def peek(self, k=0):
        return self.t[self.i + k]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, val):
        tok = self.next()
        if tok.val != val:
            raise SyntaxError(f"expected {val!r} got {tok!r}")
        return tok

    def skip_braces(self):
        """Skip a balanced {...} block starting at '{'."""
        depth = 0
        while True:
            tok = self.next()
            if tok.val == "{":
                depth += 1
            elif tok.val == "}":
                depth -= 1
                if depth == 0:
                    return

    def parse_type(self):
        """Parse a type expression; returns its textual form."""
        tok = self.peek()
        if tok.val == "[":
            self.next()
            self.expect("]")
            return "[]" + self.parse_type()
        if tok.val == "map":
            self.next()
            self.expect("[")
            k = self.parse_type()
            self.expect("]")
            return f"map[{k}]" + self.parse_type()
        if tok.val == "*":
            self.next()
            return "*" + self.parse_type()
        if tok.val == "struct":
            self.next()
            self.skip_braces()
            return "struct"
        name = self.next().val
        while self.peek().val == "." and self.peek(1).kind == "ident":
            self.next()
            name += "." + self.next().val
        return name

    def parse_expr(self):
        tok = self.peek()
        if tok.val in ("&", "*"):
            self.next()
            return Unary(tok.val, self.parse_expr())
        if tok.val == "-":
            self.next()
            x = self.parse_expr()
            return Lit(-x.v)
        return self.parse_postfix(self.parse_primary())

    def parse_primary(self):
        tok = self.peek()
        if tok.kind == "str":
            self.next()
            return Lit(tok.val)
        if tok.kind == "num":
            self.next()
            return Lit(int(tok.val) if "." not in tok.val else float(tok.val))
        if tok.val == "func":
            line = tok.line
            self.next()
            # signature up to body
            depth = 0
            while True:
                t = self.peek()
                if t.val == "(":
                    depth += 1
                elif t.val == ")":
                    depth -= 1
                elif t.val == "{" and depth == 0:
                    break
                self.next()
            self.skip_braces()
            clo = Closure(line)
            if self.peek().val == "(":
                self.next()
                self.expect(")")
            return clo
        if tok.val in ("[", "map"):
            typ = self.parse_type()
            return self.parse_composite(typ, tok.line)
        if tok.val == "(":
            self.next()
            e = self.parse_expr()
            self.expect(")")
            return e
        if tok.kind == "ident":
            self.next()
            name = tok.val
            if name in GO_PACKAGES and self.peek().val == "." and self.peek(1).kind == "ident":
                # qualified identifier (pkg.Name)
                self.next()
                name += "." + self.next().val
            if self.peek().val == "{" and (name[:1].isupper() or "." in name):
                return self.parse_composite(name, tok.line)
            return Name(name, tok.line)
        raise SyntaxError(f"unexpected {tok!r}")

    def parse_composite(self, typ, line):
        self.expect("{")
        elems = []
        while self.peek().val != "}":
            if self.peek().val == "{":
                val = self.parse_composite(None, self.peek().line)
                key = None
            else:
                first = self.parse_expr()
                if self.peek().val == ":":
                    self.next()
                    key = first
                    if self.peek().val == "{":
                        val = self.parse_composite(None, self.peek().line)
                    else:
                        val = self.parse_expr()
                else:
                    key, val = None, first
            elems.append((key, val))
            if self.peek().val == ",":
                self.next()
        self.expect("}")
        return Composite(typ, elems, line)

    def parse_args(self):
        self.expect("(")
        args = []
        while self.peek().val != ")":
            args.append(self.parse_expr())
            if self.peek().val == "...":
                self.next()
            if self.peek().val == ",":
                self.next()
        self.expect(")")
        return args

    def parse_postfix(self, x):
        while True:
            tok = self.peek()
            if tok.val == "(":
                x = Call(x, self.parse_args(), tok.line)
            elif tok.val == "." and self.peek(1).kind == "ident":
                self.next()
                name = self.next().val
                if self.peek().val == "(":
                    x = Method(x, name, self.parse_args(), tok.line)
                else:
                    x = Method(x, name, None, tok.line)
            else:
                return x


# ----------------------------------------------------------------------------
# Quantities (k8s.io/apimachinery resource.Quantity subset)
# ----------------------------------------------------------------------------
_SUFFIX = {
    "": Fraction(1), "m": Fraction(1, 1000), "k": Fraction(10**3), "M": Fraction(10**6),
    "G": Fraction(10**9), "T": Fraction(10**12), "P": Fraction(10**15), "E": Fraction(10**18),
    "Ki": Fraction(2**10), "Mi": Fraction(2**20), "Gi": Fraction(2**30), "Ti": Fraction(2**40),
    "Pi": Fraction(2**50), "Ei": Fraction(2**60),
}


def parse_quantity(s: str) -> Fraction:
    m = re.fullmatch(r"([+-]?\d+(?:\.\d*)?|[+-]?\.\d+)([a-zA-Z]*)(?:[eE]([+-]?\d+))?", s)
    if not m:
        raise ValueError(f"bad quantity {s!r}")
    num = Fraction(m.group(1))
    suf = m.group(2)
    if m.group(3) is not None:
        return num * Fraction(10) ** int(m.group(3))
    return num * _SUFFIX[suf]


def resource_value(name: str, q: Fraction) -> int:
    """resources.ResourceValue: cpu -> MilliValue, else Value (both round up)."""
    if name == "cpu":
        return math.ceil(q * 1000)
    return math.ceil(q)


class Quantity:
    def __init__(self, s):
        self.s = s
        self.q = parse_quantity(s)


# ----------------------------------------------------------------------------
# Evaluator
# ----------------------------------------------------------------------------
CONSTS = {
    "corev1.ResourceCPU": "cpu",
    "corev1.ResourceMemory": "memory",
    "corev1.ResourcePods": "pods",
    "corev1.ResourceEphemeralStorage": "ephemeral-storage",
    "corev1.LabelHostname": "kubernetes.io/hostname",
    "corev1.TaintEffectNoSchedule": "NoSchedule",
    "corev1.TaintEffectNoExecute": "NoExecute",
    "corev1.TaintEffectPreferNoSchedule": "PreferNoSchedule",
    "corev1.TolerationOpEqual": "Equal",
    "corev1.TolerationOpExists": "Exists",
    "corev1.TolerationOpLt": "Lt",
    "corev1.TolerationOpGt": "Gt",
    "corev1.NodeReady": "Ready",
    "corev1.NodeNetworkUnavailable": "NetworkUnavailable",
    "corev1.NodeMemoryPressure": "MemoryPressure",
    "corev1.NodeDiskPressure": "DiskPressure",
    "corev1.ConditionTrue": "True",
    "corev1.ConditionFalse": "False",
    "corev1.ConditionUnknown": "Unknown",
    "corev1.PodRunning": "Running",
    "corev1.PodPending": "Pending",
    "corev1.PodSucceeded": "Succeeded",
    "corev1.PodFailed": "Failed",
    "true": True,
    "false": False,
    "nil": None,
    "features.TASProfileMixed": "TASProfileMixed",
    "features.TASBalancedPlacement": "TASBalancedPlacement",
    "features.TASMultiLayerTopology": "TASMultiLayerTopology",
    "features.ElasticJobsViaWorkloadSlicesWithTAS": "ElasticJobsViaWorkloadSlicesWithTAS",
    "features.TASFailedNodeReplacement": "TASFailedNodeReplacement",
    "features.ElasticJobsViaWorkloadSlices": "ElasticJobsViaWorkloadSlices",
    "features.TASFailedNodeReplacementFailFast": "TASFailedNodeReplacementFailFast",
}


class Unsupported(Exception):
    pass


class NodeB:
    def __init__(self, name):
        self.d = {"name": name, "labels": {}, "allocatable": {}, "taints": [],
                  "unschedulable": False, "conditions": []}

    def call(self, m, args):
        d = self.d
        if m == "Label":
            d["labels"][args[0]] = args[1]
        elif m == "StatusAllocatable":
            for k, v in args[0].items():
                d["allocatable"][k] = resource_value(k, v.q)
        elif m == "Ready":
            d["conditions"].append({"type": "Ready", "status": "True"})
        elif m == "NotReady":
            d["conditions"].append({"type": "Ready", "status": "False"})
        elif m == "Unschedulable":
            d["unschedulable"] = True
        elif m == "Taints":
            d["taints"].extend(args)
        elif m == "StatusConditions":
            d["conditions"].extend({"type": c.get("Type", ""), "status": c.get("Status", "")} for c in args)
        elif m == "Obj":
            return self
        else:
            raise Unsupported(f"node method {m}")
        return self


class PodB:
    def __init__(self, name, ns):
        self.d = {"name": name, "namespace": ns, "nodeName": "", "phase": "", "requests": {}}

    def call(self, m, args):
        d = self.d
        if m == "NodeName":
            d["nodeName"] = args[0]
        elif m == "StatusPhase":
            d["phase"] = args[0]
        elif m == "Request":
            d["requests"][args[0]] = resource_value(args[0], parse_quantity(args[1]))
        elif m == "Obj":
            return self
        else:
            raise Unsupported(f"pod method {m}")
        return self


def _taint(d):
    return {"key": d.get("Key", ""), "value": d.get("Value", ""), "effect": d.get("Effect", "")}


def _toleration(d):
    return {"key": d.get("Key", ""), "operator": d.get("Operator", ""), "value": d.get("Value", ""),
            "effect": d.get("Effect", "")}


class Evaluator:
    def __init__(self, env):
        self.env = env

    def ev(self, x, typ_hint=None):
        if isinstance(x, Lit):
            return x.v
        if isinstance(x, Name):
            if x.n in self.env:
                return self.env[x.n]
            if x.n in CONSTS:
                return CONSTS[x.n]
            raise Unsupported(f"name {x.n} (line {x.line})")
        if isinstance(x, Unary):
            return self.ev(x.x, typ_hint)
        if isinstance(x, Closure):
            if x.line in CLOSURES:
                return CLOSURES[x.line]()
            raise Unsupported(f"closure at line {x.line}")
        if isinstance(x, Call):
            fn = x.fn.n if isinstance(x.fn, Name) else None
            args = [self.ev(a) for a in x.args]
            if fn in ("ptr.To", "new"):
                return args[0]
            if fn == "append":
                return list(args[0]) + [a for extra in args[1:] for a in (extra if isinstance(extra, list) else [extra])]
            if fn in ("int32", "int64", "int", "string", "corev1.ResourceName", "kueue.PodSetReference",
                      "kueue.TopologyReference"):
                return args[0]
            if fn == "tas.V1Beta2From":
                # previousAssignment (v1beta2); the fixture keeps the internal
                # form: InternalFrom(V1Beta2From(x)) == x (pinned by the
                # encoding goldens, tests/golden/tas_v1beta2_encoding.json)
                return args[0]
            if fn == "resource.MustParse":
                return Quantity(args[0])
            if fn == "testingnode.MakeNode":
                return NodeB(args[0])
            if fn == "testingpod.MakePod":
                return PodB(args[0], args[1])
            raise Unsupported(f"call {fn} (line {x.line})")
        if isinstance(x, Method):
            recv = self.ev(x.recv)
            args = [self.ev(a) for a in (x.args or [])]
            if isinstance(recv, (NodeB, PodB)):
                return recv.call(x.name, args)
            raise Unsupported(f"method {x.name} on {type(recv).__name__} (line {x.line})")
        if isinstance(x, Composite):
            return self.composite(x, typ_hint)
        raise Unsupported(f"node {type(x).__name__}")

    def composite(self, c, typ_hint):
        typ = c.typ if c.typ is not None else typ_hint
        if typ is None:
            raise Unsupported(f"untyped composite at line {c.line}")
        if typ.startswith("[]"):
            elem_t = typ[2:]
            return [self.ev(v, elem_t) for _, v in c.elems]
        if typ.startswith("map["):
            out = {}
            val_t = typ[typ.index("]") + 1:]
            for k, v in c.elems:
                out[self.ev(k)] = self.ev(v, val_t)
            return out
        if typ == "struct":
            raise Unsupported("anonymous struct literal")
        if typ in MAP_TYPES:
            return {self.ev(k): self.ev(v) for k, v in c.elems}
        fields = {}
        for k, v in c.elems:
            if not isinstance(k, Name):
                raise Unsupported(f"positional struct literal {typ} at line {c.line}")
            fields[k.n] = self.ev(v, FIELD_TYPES.get((typ, k.n)))
        if typ in ("corev1.ResourceList", "resources.Requests"):
            return fields
        if typ == "corev1.Taint":
            return _taint(fields)
        if typ == "corev1.Toleration":
            return _toleration(fields)
        return fields


MAP_TYPES = {"corev1.ResourceList", "resources.Requests"}

FIELD_TYPES = {
    ("kueue.PodSetTopologyRequest", "PodsetSliceRequiredTopologyConstraints"):
        "[]kueue.PodsetSliceRequiredTopologyConstraint",
    ("tas.TopologyAssignment", "Domains"): "[]tas.TopologyDomainAssignment",
    ("PodSetTestCase", "wantAssignment"): "*tas.TopologyAssignment",
    ("PodSetTestCase", "previousAssignment"): "*tas.TopologyAssignment",
}


# The only closure-built node set in the table (tas_cache_test.go:5890-5922) is
# transcribed here: 8 racks x 18 nodes, 2 nvidia.com/gpu + 110 pods each.
def _gb200_nodes():
    racks = [
        ("dc0", "aizone0", "block0", "r0"), ("dc0", "aizone0", "block0", "r1"),
        ("dc0", "aizone0", "block1", "r2"), ("dc0", "aizone0", "block1", "r3"),
        ("dc0", "aizone1", "block2", "r4"), ("dc0", "aizone1", "block2", "r5"),
        ("dc0", "aizone1", "block3", "r6"), ("dc0", "aizone1", "block3", "r7"),
    ]
    out = []
    for dc, az, block, rack in racks:
        for i in range(18):
            n = NodeB(f"{block}-{rack}-{az}-n{i}")
            n.call("Label", ["cloud.com/datacenter", dc])
            n.call("Label", ["cloud.com/aizone", az])
            n.call("Label", ["cloud.com/topology-block", block])
            n.call("Label", ["cloud.com/topology-rack", rack])
            n.d["allocatable"] = {"nvidia.com/gpu": 2, "pods": 110}
            n.call("Ready", [])
            out.append(n)
    return out


CLOSURES = {}


def _find(toks, seq, start=0):
    n = len(seq)
    for i in range(start, len(toks) - n):
        if all(toks[i + j].val == seq[j] for j in range(n)):
            return i
    raise ValueError(f"sequence {seq} not found")


def _to_json_node(n):
    d = dict(n.d)
    d["taints"] = list(d["taints"])
    return d


def normalise_case(name, line, raw):
    """Turn an evaluated case struct into the fixture schema."""
    out = {"name": name, "line": line, "scope": "in"}
    fg = raw.get("featureGates") or {}
    out["featureGates"] = fg
    out["levels"] = raw.get("levels") or []
    out["nodeLabels"] = raw.get("nodeLabels") or {}
    out["nodes"] = [_to_json_node(n) for n in raw.get("nodes") or []]
    out["pods"] = [p.d for p in raw.get("pods") or []]
    pss = []
    for ps in raw.get("podSets") or []:
        tr = ps.get("topologyRequest")
        if tr is not None:
            tr = {
                "required": tr.get("Required"),
                "preferred": tr.get("Preferred"),
                "unconstrained": tr.get("Unconstrained"),
                "podSetSliceRequiredTopology": tr.get("PodSetSliceRequiredTopology"),
                "podSetSliceSize": tr.get("PodSetSliceSize"),
                "podsetSliceRequiredTopologyConstraints": [
                    {"topology": c["Topology"], "size": c["Size"]}
                    for c in (tr.get("PodsetSliceRequiredTopologyConstraints") or [])
                ],
                "podSetGroupName": None,
            }
        wa = ps.get("wantAssignment")
        if wa is not None:
            wa = {"levels": wa.get("Levels") or [],
                  "domains": [{"values": d.get("Values") or [], "count": d.get("Count", 0)}
                              for d in (wa.get("Domains") or [])]}
        pa = ps.get("previousAssignment")
        if pa is not None:
            pa = {"levels": pa.get("Levels") or [],
                  "domains": [{"values": d.get("Values") or [], "count": d.get("Count", 0)}
                              for d in (pa.get("Domains") or [])]}
        pss.append({
            "name": (ps.get("podSetName") or "").lower(),
            "topologyRequest": tr,
            "requests": ps.get("requests") or {},
            "count": ps.get("count", 0),
            "tolerations": ps.get("tolerations") or [],
            "nodeSelector": ps.get("nodeSelector"),
            "podSetGroupName": ps.get("podSetGroupName"),
            "wantAssignment": wa,
            "wantReason": ps.get("wantReason") or "",
            **({"previousAssignment": pa} if pa is not None else {}),
        })
    out["podSets"] = pss
    return out


def extract(ref_root):
    src = open(os.path.join(ref_root, REF_TEST)).read()
    toks = tokenize(src)
    fn = _find(toks, ["func", "TestFindTopologyAssignments", "("])
    env = {}
    CLOSURES.clear()
    # constants block: const ( name = "..." ... )
    i = _find(toks, ["const", "("], fn)
    j = i + 2
    while toks[j].val != ")":
        env[toks[j].val] = toks[j + 2].val
        j += 3
    # closure line for the GB200 set
    for t in toks[fn:]:
        if t.val == "func" and t.line > 5850:
            CLOSURES[t.line] = _gb200_nodes
            break
    # shared variables: name := expr   (until `cases :=`)
    cases_at = _find(toks, ["cases", ":="], fn)
    k = j
    while k < cases_at:
        if toks[k].kind == "ident" and toks[k + 1].val == ":=":
            p = Parser(toks, k + 2)
            expr = p.parse_expr()
            env[toks[k].val] = Evaluator(env).ev(expr)
            k = p.i
        else:
            k += 1
    # the cases map literal
    p = Parser(toks, cases_at + 2)
    p.parse_type()  # map[string]struct{...}
    p.expect("{")
    cases = []
    while p.peek().val != "}":
        name_tok = p.next()
        assert name_tok.kind == "str", name_tok
        p.expect(":")
        body = p.parse_composite("case", name_tok.line)
        if p.peek().val == ",":
            p.next()
        ev = Evaluator(env)
        raw = {}
        err = None
        for key, val in body.elems:
            try:
                raw[key.n] = ev.ev(val)
            except Unsupported as e:  # noqa: PERF203
                err = str(e)
        if err is not None:
            cases.append({"name": name_tok.val, "line": name_tok.line, "scope": f"out:unparsed ({err})"})
            continue
        cases.append(normalise_case(name_tok.val, name_tok.line, raw))
    return cases


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(__file__), "..", "tests", "golden", "tas_find_topology_assignments.json")
    cases = extract(ref)
    doc = {
        "source": f"{REF_TEST} TestFindTopologyAssignments (reference :55-6341)",
        "generator": "tools/extract_goldens.py",
        "cases": cases,
    }
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=False)
        f.write("\n")
    n_in = sum(1 for c in cases if c["scope"] == "in")
    print(f"wrote {len(cases)} cases ({n_in} in scope) -> {out}")
    for c in cases:
        if c["scope"] != "in":
            print(f"  L{c['line']}: {c['scope']}: {c['name']}")


if __name__ == "__main__":
    main()
