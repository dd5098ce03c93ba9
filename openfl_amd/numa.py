"""Host NUMA placement for a GPU process.

A GPU's PCIe link hangs off one socket.  Host buffers the pipelines touch on
every call -- the payload `bytes` the device gzip fills, the pinned staging
of the payload's H2D, the serial seed sum's threads -- run at the local
socket's memory and PCIe rate only when the threads that first touch them
run on that socket.  Measured on a two-socket MI355X host whose process may
run on any CPU (profiles/r06_env_ab.txt, bench.py alternated, HIP's 4 and
8 HW queues): the KC pipeline runs 50.5-52.3 GiB/s bound against 46.8-49.9
unbound, the gzip and inflate phases carrying the difference; the
device-resident Eden step does not gain (422-425 GiB/s bound, 425-438
unbound).  bench.py therefore runs on the OS placement and measures the KC
steps bound in a child process beside it (numa_bound_variant).

bind_to_device(i) restricts every thread of the process (and the threads it
starts later) to the CPUs of the GPU's NUMA node, within the CPUs the process
is allowed; memory first touched afterwards is then node-local.  It is
process-wide, so the framework never calls it by itself: tools/kc_bench.py
and bench.py --numa-bind call it, and a deployment that runs the host-heavy
lossy pipelines calls it once per process after choosing the device (the
equivalent of `numactl --cpunodebind`)."""
import os

__all__ = ["device_numa_node", "bind_to_device"]


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpulist(text):
    cpus = set()
    for part in (text or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def device_numa_node(index):
    """NUMA node of torch device `index` (its PCI function's sysfs
    numa_node), or None when the platform does not say."""
    import torch
    p = torch.cuda.get_device_properties(index)
    bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}.0"
    node = _read(f"/sys/bus/pci/devices/{bdf}/numa_node")
    if node is None or int(node) < 0:
        return None
    return int(node)


def bind_to_device(index):
    """Bind every thread of this process to the CPUs of device `index`'s NUMA
    node (within the allowed CPUs).  Returns the CPU list, or None when the
    node or its CPUs are unknown (nothing changed)."""
    node = device_numa_node(index)
    if node is None:
        return None
    cpus = _cpulist(_read(f"/sys/devices/system/node/node{node}/cpulist")) & os.sched_getaffinity(0)
    if not cpus:
        return None
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:  # a thread that exited meanwhile
            pass
    return sorted(cpus)
