// device_filters.h — the default-profile filter chain on the mirror's SoA rows
// (SF/runtime/framework.go:727-749; plugin order default_plugins.go:33-53).
// Cold rows (NodeStatic / NodeExt) are touched only when the pod or the node
// needs them, so a resource-only evaluation reads one 32-B NodeHot row.
#pragma once
#include "casim_internal.h"

namespace casim {

__device__ inline int dev_full_filters(const ca_pod_spec& s, const PodHot& p, const ca_selector_term* terms,
                                       const ca_selector_req* reqs, const NodeHot& h,
                                       const NodeExt* __restrict__ ext, const NodeStatic* __restrict__ st,
                                       bool apply_unsched, uint32_t* reasons) {
    *reasons = 0;
    if (apply_unsched && (h.flags & NF_UNSCHED) && !(p.flags & PF_TOL_UNSCHED))
        return CA_PLUGIN_NODE_UNSCHEDULABLE;                                 // node_unschedulable.go:61-75
    const bool need_static = (p.flags & (PF_NODE_NAME | PF_AFFINITY)) ||
                             ((h.flags & NF_TAINTS) && !(p.flags & PF_TAINT_MASK_ALL));
    if (need_static) {
        const NodeStatic ns = *st;
        const int pl = dev_static_filters(s, p.flags, terms, reqs, ns, false);
        if (pl != CA_PLUGIN_NONE) return pl;
    }
    int64_t fsc[CA_MAX_SCALAR];
    const bool need_ext = ((p.flags & PF_PORTS) && (h.flags & NF_PORTS)) || (p.flags & PF_SCALAR_REQ);
    if (need_ext) {
        const NodeExt ne = *ext;
        if (p.flags & PF_PORTS) {                                             // node_ports.go:117-141
            uint64_t c = 0;
            for (int w = 0; w < CA_PORT_WORDS; w++) c |= ne.ports[w] & s.port_conflict[w];
            if (c) return CA_PLUGIN_NODE_PORTS;
        }
        for (int i = 0; i < CA_MAX_SCALAR; i++) fsc[i] = ne.scalar[i];
    } else {
        for (int i = 0; i < CA_MAX_SCALAR; i++) fsc[i] = 0;
    }
    const uint32_t r = dev_fit_reasons(p.cpu, p.mem, p.eph, p.flags, s.req_scalar, h.cpu, h.mem, h.eph, h.pods, fsc);
    if (r) { *reasons = r; return CA_PLUGIN_NODE_RESOURCES_FIT; }
    return CA_PLUGIN_NONE;
}

}  // namespace casim
