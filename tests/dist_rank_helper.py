"""One rank of the CPU stand-in for bench.py's N-rank path, started by
bench.launch_ranks (torch.distributed.run in a child process) from
tests/test_bench_launch.py: a gloo process group, the rank's interleaved row
tiles rendered by the fp32 oracle (standing in for rtx_render_rows — test
infrastructure, no GPU), one gather to rank 0 (rtx/dist.py FrameGather, the
class bench.py drives over RCCL), the host de-interleave. Rank 0 saves the
frame and what the launcher handed the ranks (env and world size).

    helper.py OUT_DIR W H T SPP
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytrace-we-gpu_amd"), os.path.join(ROOT, "oracle")]


def main():
    out, W, H, T, spp = sys.argv[1], *map(int, sys.argv[2:6])
    import numpy as np
    import torch
    import torch.distributed as dist

    import oracle
    import rtx
    from rtx.dist import FrameGather, part_row_ids

    dist.init_process_group("gloo")
    rank, R = dist.get_rank(), dist.get_world_size()
    world = rtx.random_world(4, depth=20, spp=spp)
    frame = rtx.camera_look_at(W, H, aspect=W / H)

    def render_part(send, part, nparts):
        ids = part_row_ids(H, T, part, nparts)
        rows, _ = oracle.render_rows(world, frame, ids, nthreads=1)
        send[:len(ids)] = torch.from_numpy(rows)

    marks = []
    fg = FrameGather(W, H, T, rank, R, render_part)
    fg.mark = marks.append
    img = fg.step()
    seen = [None] * R
    dist.all_gather_object(seen, {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]),
                                  "world_size": int(os.environ["WORLD_SIZE"]), "marks": marks,
                                  "ipc_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"),
                                  "launched": os.environ.get("RTX_BENCH_RANKS_LAUNCHED"),
                                  "master_addr": os.environ.get("MASTER_ADDR")})
    if rank == 0:
        np.save(os.path.join(out, "img.npy"), img.numpy())
        with open(os.path.join(out, "ranks.json"), "w") as f:
            json.dump(seen, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
