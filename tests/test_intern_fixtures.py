"""Interning fixtures for a Go shim (tests/golden/intern_fixtures.json):
the Python interning reproduces every committed record, and the records carry the
reference semantics checked by hand below (toleration masks, port-conflict wildcards,
selector programs, scope flags)."""
import json
import os

from autoscaler_amd import abi

import importlib.util

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "intern_fixtures.json")))
_spec = importlib.util.spec_from_file_location("mif", os.path.join(HERE, "golden", "make_intern_fixtures.py"))
mif = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mif)


def case(name):
    return next(c for c in FIX["cases"] if c["name"].startswith(name))


def test_fixtures_reproduce():
    for c in FIX["cases"]:
        assert mif.build(c["input"]) == c["expect"], c["name"]


def test_taint_semantics():
    e = case("taints")["expect"]
    taints = [tuple(t) for t in e["universes"]["taints"]]
    # PreferNoSchedule is not a filter effect (helpers.go:78-101): not interned
    assert ("soft", "x", "PreferNoSchedule") not in taints and len(taints) == 3
    bit = {t: 1 << i for i, t in enumerate(taints)}
    tol = {p["similar_class"]: p for p in e["pods"]}   # not used; by position below
    none, exists, equal, alls, unsched = e["pods"]
    assert none["tolerated_taints"] == 0
    assert exists["tolerated_taints"] == bit[("dedicated", "ml", "NoSchedule")] | bit[("dedicated", "web", "NoSchedule")]
    assert equal["tolerated_taints"] == bit[("dedicated", "ml", "NoSchedule")]
    assert alls["tolerated_taints"] == (1 << 64) - 1 or alls["tolerated_taints"] == sum(bit.values())
    assert unsched["flags"] & abi.CA_POD_TOLERATES_UNSCHED and not exists["flags"] & abi.CA_POD_TOLERATES_UNSCHED
    assert e["nodes"][1]["flags"] & abi.CA_NODE_UNSCHEDULABLE
    del tol


def test_port_wildcards():
    e = case("host ports")["expect"]
    ports = [tuple(p) for p in e["universes"]["ports"]]
    assert ports == [("0.0.0.0", "TCP", 8080), ("10.0.0.1", "TCP", 8080), ("0.0.0.0", "UDP", 8080)]
    tcp, ip, udp = e["pods"]
    assert tcp["port_conflict"][0] == 0b011 and ip["port_conflict"][0] == 0b011 and udp["port_conflict"][0] == 0b100
    assert tcp["port_use"][0] == 0b001 and ip["port_use"][0] == 0b010


def test_selector_programs():
    e = case("node selectors")["expect"]
    sel, innotin, exists, fields, bad, hostname, node_name = e["pods"]
    assert sel["flags"] & abi.CA_POD_AFFINITY_FILTER and sel["aff_term_count"] == -1
    assert innotin["aff_term_count"] == 2
    ops = [r["op"] for r in e["reqs"]]
    assert ops[:3] == [abi.CA_OP_IN, abi.CA_OP_NOTIN, abi.CA_OP_GT]
    assert fields["flags"] & abi.CA_POD_PREFILTER_NAMES and e["prefilter_names"] == [e["universes"]["names"].index("a2")]
    # a term with an unparsable Gt/Lt value never matches; an empty term is dropped
    assert bad["aff_term_count"] == 1 and e["reqs"][e["terms"][bad["aff_term_first"]]["first"]]["op"] == abi.CA_OP_FALSE
    assert hostname["flags"] & abi.CA_POD_HOSTNAME_DEPENDENT and node_name["flags"] & abi.CA_POD_HOSTNAME_DEPENDENT
    a1, a2 = e["nodes"]
    gen = e["universes"]["int_keys"].index("gen")
    assert a1["int_label_valid"] >> gen & 1 and a1["int_label"][gen] == 5 and not a2["int_label_valid"] >> gen & 1


def test_resources_and_scope():
    e = case("resources")["expect"]
    plain, init, overhead, gpu, tpu, zero, milli = e["pods"]
    assert init["req_milli_cpu"] == 2000 and init["score_milli_cpu"] == 250          # init max; score = containers
    assert overhead["req_milli_cpu"] == 350 and overhead["score_milli_cpu"] == 250
    assert gpu["flags"] & abi.CA_POD_HAS_SCALAR_KEYS and gpu["flags"] & abi.CA_POD_HAS_NONTPU_SCALAR_KEYS
    assert tpu["flags"] & abi.CA_POD_HAS_SCALAR_KEYS and not tpu["flags"] & abi.CA_POD_HAS_NONTPU_SCALAR_KEYS
    assert tpu["tpu_scalar_mask"] != 0
    assert zero["req_milli_cpu"] == 0 and zero["req_memory"] == 0
    assert milli["req_milli_cpu"] == 1 and milli["req_memory"] == 2                   # MilliValue / Value round up
    s = case("kernel scope")["expect"]["pods"]
    flags = [p["flags"] for p in s]
    oos = [bool(f & abi.CA_POD_OUT_OF_SCOPE) for f in flags]
    assert oos == [True, False, True, True, False, False, False, False, False]
    assert flags[2] & abi.CA_POD_REQUIRED_ANTI_AFFINITY
    assert flags[5] & abi.CA_POD_DAEMONSET and flags[6] & abi.CA_POD_DAEMONSET
    assert s[7]["similar_class"] == s[8]["similar_class"] >= 0
