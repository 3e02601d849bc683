"""Seeded random clusters exercising every in-kernel filter: taints/tolerations,
nodeSelector, required node affinity (In/NotIn/Exists/DoesNotExist/Gt/Lt,
matchFields), host ports (wildcard and specific IPs), extended resources,
unschedulable nodes, zero-request pods, init containers and overhead."""
from __future__ import annotations

import random

from autoscaler_amd import k8s
from autoscaler_amd.k8s import (Affinity, Container, ContainerPort, Node, NodeSelectorRequirement, NodeSelectorTerm,
                                OwnerReference, Pod, Quantity, Taint, Toleration)

ZONES = ["z1", "z2", "z3"]
TIERS = ["gold", "silver", "bronze"]
TAINTS = [("dedicated", "batch", "NoSchedule"), ("dedicated", "web", "NoSchedule"), ("gpu", "present", "NoSchedule"),
          ("spot", "true", "NoExecute"), ("soft", "x", "PreferNoSchedule")]
EXT = ["example.com/fpga", "nvidia.com/gpu"]


def rand_node(rng: random.Random, name: str, big: bool = False) -> Node:
    cpu = rng.choice([1000, 2000, 4000, 8000]) * (4 if big else 1)
    mem = rng.choice([2, 4, 8, 16]) * (1 << 30) * (4 if big else 1)
    n = k8s.build_test_node(name, cpu, mem, rng.choice([5, 10, 110]))
    if rng.random() < 0.3:
        n.allocatable["ephemeral-storage"] = Quantity(rng.choice([10, 20]) * (1 << 30))
    n.labels["zone"] = rng.choice(ZONES)
    if rng.random() < 0.7:
        n.labels["tier"] = rng.choice(TIERS)
    if rng.random() < 0.6:
        n.labels["rank"] = str(rng.randint(-5, 20)) if rng.random() < 0.9 else "NaN"
    if rng.random() < 0.3:
        n.taints.append(Taint(*rng.choice(TAINTS)))
    if rng.random() < 0.2:
        n.allocatable[rng.choice(EXT)] = Quantity(rng.randint(0, 4))
    n.unschedulable = rng.random() < 0.1
    return n


def rand_pod(rng: random.Random, name: str, small: bool = False) -> Pod:
    cpu = rng.choice([0, 100, 250, 500, 1000, 2000]) // (4 if small else 1)
    mem = rng.choice([0, 128, 512, 1024, 4096]) * (1 << 20) // (4 if small else 1)
    p = k8s.build_test_pod(name, cpu, mem)
    if rng.random() < 0.15:
        p.containers.append(Container(requests={"cpu": Quantity.milli(rng.choice([0, 50, 100]))}))
    if rng.random() < 0.1:
        p.init_containers.append(Container(requests={"cpu": Quantity.milli(rng.choice([100, 3000]))}))
    if rng.random() < 0.05:
        p.overhead = {"cpu": Quantity.milli(50)}
    if rng.random() < 0.1:
        p.containers[0].requests[rng.choice(EXT)] = Quantity(rng.choice([0, 1, 2]))
    if rng.random() < 0.1:
        p.containers[0].requests["ephemeral-storage"] = Quantity(rng.choice([1, 5]) * (1 << 30))
    if rng.random() < 0.15:
        p.containers[0].ports.append(ContainerPort(host_port=rng.choice([80, 443, 8080]),
                                                   host_ip=rng.choice(["", "", "10.0.0.1", "10.0.0.2"]),
                                                   protocol=rng.choice(["", "TCP", "UDP"])))
    if rng.random() < 0.4:
        for _ in range(rng.randint(1, 2)):
            t = rng.choice(TAINTS)
            p.tolerations.append(rng.choice([
                Toleration(key=t[0], operator="Equal", value=t[1], effect=t[2]),
                Toleration(key=t[0], operator="Exists"),
                Toleration(operator="Exists"),
                Toleration(key=t[0], operator="Equal", value="other"),
                Toleration(key="node.kubernetes.io/unschedulable", operator="Exists", effect="NoSchedule"),
            ]))
    if rng.random() < 0.3:
        p.node_selector = {"zone": rng.choice(ZONES)} if rng.random() < 0.8 else {}
    if rng.random() < 0.3:
        terms = []
        for _ in range(rng.randint(0, 2)):
            exprs = []
            for _ in range(rng.randint(0, 2)):
                op = rng.choice(["In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt", "Bogus"])
                key = rng.choice(["zone", "tier", "rank", "missing"])
                if op in ("In", "NotIn"):
                    vals = rng.sample(ZONES + TIERS, rng.randint(0, 2))
                elif op in ("Gt", "Lt"):
                    vals = [str(rng.randint(-3, 15))] if rng.random() < 0.9 else ["x"]
                else:
                    vals = []
                exprs.append(NodeSelectorRequirement(key, op, vals))
            fields = []
            if rng.random() < 0.1:
                fields.append(NodeSelectorRequirement("metadata.name", rng.choice(["In", "NotIn"]),
                                                      [f"n{rng.randint(0, 6)}"]))
            terms.append(NodeSelectorTerm(exprs, fields))
        p.affinity = Affinity(required_terms=terms)
    if rng.random() < 0.05:
        p.node_name = f"n{rng.randint(0, 6)}"
    if rng.random() < 0.5:
        p.owner_refs = [OwnerReference("ReplicaSet", f"rs{rng.randint(0, 3)}", f"rs{rng.randint(0, 3)}")]
    return p


def rand_cluster(seed: int, n_nodes: int = 8, n_pods: int = 24, pods_per_node: int = 3):
    rng = random.Random(seed)
    nodes = [rand_node(rng, f"n{i}") for i in range(n_nodes)]
    scheduled = []
    for i in range(min(n_pods, n_nodes * pods_per_node)):
        p = rand_pod(rng, f"s{i}", small=True)
        p.node_name = ""
        p.affinity = None
        p.node_selector = None
        scheduled.append((p, nodes[i % n_nodes].name))
    pending = [rand_pod(rng, f"p{i}") for i in range(n_pods)]
    return rng, nodes, scheduled, pending
