"""Diagnostic: CPU affinity of the main thread and the process's threads before and after an
RCCL process group is created (one rank, launched under torch.distributed.run)."""
import os
import threading
import time

import torch
import torch.distributed as dist


def show(tag):
    tids = os.listdir("/proc/self/task")
    aff = {}
    for t in tids:
        try:
            aff[t] = len(os.sched_getaffinity(int(t)))
        except OSError:
            pass
    print(tag, "main affinity", len(os.sched_getaffinity(0)), "threads", len(tids), "thread affinities", sorted(set(aff.values())),
          flush=True)


show("before")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
dist.barrier()
time.sleep(0.5)
show("after")
# a spinning main thread: how many busy threads compete?
import subprocess
print(subprocess.run(["ps", "-L", "-o", "tid,psr,pcpu,comm", "-p", str(os.getpid())], capture_output=True, text=True).stdout,
      flush=True)
dist.destroy_process_group()
