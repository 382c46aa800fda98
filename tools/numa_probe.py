"""Host -> device upload rate by the host pages' NUMA node (the whole-file GPU decode uploads a
page-locked copy of the file; where those pages live decides its PCIe rate).  For every NUMA node
this process may run on: pin the thread to that node's CPUs, first-touch a buffer (pages land on
the node), page-lock it (hipHostRegister), time H2D copies; then the same for hipHostMalloc memory
(torch pin_memory).  Measurements only.

  python tools/numa_probe.py [MiB]
"""
import glob
import json
import os
import re
import sys
import time

import numpy as np
import torch


def cpu_node():
    m = {}
    for d in glob.glob("/sys/devices/system/cpu/cpu[0-9]*"):
        cpu = int(re.findall(r"\d+$", d)[0])
        nodes = glob.glob(d + "/node*")
        m[cpu] = int(re.findall(r"\d+$", nodes[0])[0]) if nodes else 0
    return m


def gpu_node():
    for p in sorted(glob.glob("/sys/class/drm/card*/device/numa_node")):
        try:
            return int(open(p).read())
        except OSError:
            pass
    return None


def rate(src, dst, reps=10):
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return src.numel() * reps / (time.perf_counter() - t) / 1e9


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    dev = torch.device("cuda", 0)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    allowed = sorted(os.sched_getaffinity(0))
    cn = cpu_node()
    by_node = {}
    for c in allowed:
        by_node.setdefault(cn.get(c, 0), []).append(c)
    rt = torch.cuda.cudart()
    rows = []
    for node, cpus in sorted(by_node.items()):
        os.sched_setaffinity(0, cpus)
        buf = np.ones(n, dtype=np.uint8)  # first touch on this node's CPUs
        rc = rt.cudaHostRegister(buf.ctypes.data, n, 0)
        src = torch.from_numpy(buf)
        r = {"kind": "registered", "first_touch_node": node, "cpus": len(cpus), "register_rc": int(rc),
             "h2d_GBps": round(rate(src, dst), 2)}
        rt.cudaHostUnregister(buf.ctypes.data)
        rows.append(r)
        print(json.dumps(r), flush=True)
    os.sched_setaffinity(0, allowed)
    pm = torch.empty(n, dtype=torch.uint8).pin_memory()
    r = {"kind": "hipHostMalloc", "h2d_GBps": round(rate(pm, dst), 2)}
    print(json.dumps(r), flush=True)
    print(json.dumps({"gpu_numa_node": gpu_node(), "nodes_allowed": sorted(by_node), "numa_nodes":
                      len(glob.glob("/sys/devices/system/node/node[0-9]*"))}), flush=True)


if __name__ == "__main__":
    main()
