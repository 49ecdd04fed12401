"""Launcher probe for tests/test_dist.py: `python tests/dist_probe.py --gpus N` started as one process must
come back as N ranks (3dgvrt_lightfield_amd.dist.launch_ranks, the launcher bench.py uses); each rank joins a
gloo group and rank 0 prints the group's size.  CPU only."""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--gpus", type=int, default=1)
args = ap.parse_args()
d = importlib.import_module("3dgvrt_lightfield_amd.dist")
rc = d.launch_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:])
if rc is not None:
    sys.exit(rc)
import torch.distributed as dist  # noqa: E402

world = int(os.environ.get("WORLD_SIZE", "1"))
if world > 1:
    dist.init_process_group("gloo")
    world = dist.get_world_size()
if int(os.environ.get("RANK", "0")) == 0:
    print(json.dumps({"n_gpus": world, "gpus_arg": args.gpus}), flush=True)
if world > 1:
    dist.barrier()
    dist.destroy_process_group()
