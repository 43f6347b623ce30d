"""Process-group setup for the multi-process GPU tests: RCCL (backend
"nccl") with one device per rank when the box has at least `ws` GPUs, gloo
over one shared device otherwise (the 1-GPU test boxes)."""
import datetime

import torch
import torch.distributed as dist


def init_gpu_group(rank: int, ws: int, timeout_s: int = 300) -> torch.device:
    # device_count() does not initialise the GPU on this image
    multi = torch.cuda.device_count() >= ws
    to = datetime.timedelta(seconds=timeout_s)
    if multi:
        dev = torch.device("cuda", rank)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=ws, timeout=to, device_id=dev)
    else:
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=ws, timeout=to)
    return dev
