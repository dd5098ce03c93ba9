"""Host topology seen by this process on the GPU box: allowed CPUs, NUMA
nodes and their CPUs, the GPU's PCI NUMA node, memory per node.  Prints JSON."""
import glob
import json
import os


def rd(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.__class__.__name__}>"


def main():
    out = {"allowed_cpus": sorted(os.sched_getaffinity(0))}
    out["nodes"] = {os.path.basename(n): rd(os.path.join(n, "cpulist"))
                    for n in sorted(glob.glob("/sys/devices/system/node/node[0-9]*"))}
    gpus = {}
    for d in sorted(glob.glob("/sys/class/drm/card[0-9]*/device")):
        gpus[d] = {"numa_node": rd(os.path.join(d, "numa_node")), "vendor": rd(os.path.join(d, "vendor")),
                   "uevent_pci": [l for l in rd(os.path.join(d, "uevent")).splitlines() if l.startswith("PCI_SLOT")]}
    out["drm"] = gpus
    out["visible"] = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    out["mems_allowed"] = [l for l in rd("/proc/self/status").splitlines() if l.startswith(("Cpus_allowed_list", "Mems_allowed_list"))]
    try:
        import torch
        p = torch.cuda.get_device_properties(0)
        out["torch_pci"] = {"bus": getattr(p, "pci_bus_id", None), "domain": getattr(p, "pci_domain_id", None),
                            "device": getattr(p, "pci_device_id", None), "name": p.name}
    except Exception as e:  # noqa: BLE001
        out["torch_pci"] = repr(e)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
