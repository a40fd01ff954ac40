"""Where the GPU box's visible GPU sits relative to this process: the render
nodes the box exposes, each one's NUMA node and local CPUs (sysfs), and the
CPUs this process may run on.  Used to diagnose the host-memory (e2e) leg's
box-to-box spread."""
import glob
import json
import os


def read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return "unreadable: %s" % e.__class__.__name__


out = {"affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "dri": sorted(os.listdir("/dev/dri")) if os.path.isdir("/dev/dri") else None}
nodes = []
for r in sorted(glob.glob("/sys/class/drm/renderD*")):
    dev = os.path.join(r, "device")
    nodes.append({"node": os.path.basename(r), "in_dev": os.path.exists("/dev/dri/" + os.path.basename(r)),
                  "numa_node": read(os.path.join(dev, "numa_node")), "local_cpulist": read(os.path.join(dev, "local_cpulist")),
                  "pci": os.path.basename(os.path.realpath(dev))})
out["render"] = nodes
out["numa_nodes"] = {os.path.basename(n): read(os.path.join(n, "cpulist")) for n in sorted(glob.glob("/sys/devices/system/node/node*"))}
out["hip_visible"] = os.environ.get("HIP_VISIBLE_DEVICES"), os.environ.get("ROCR_VISIBLE_DEVICES")
print(json.dumps(out, indent=1))
