#!/usr/bin/env python3
"""Round 5: the row-slab gather forms over gloo with CPU tensors, two ranks:
batch_isend_irecv of the exact slabs to rank 0 vs an all-gather of padded slabs, 4096^2
fp32.  (Over gloo with CUDA tensors the point-to-point form costs ~1.2-1.4 s per map.)"""
import os, time, torch, torch.distributed as dist
import torch.multiprocessing as mp
def run(rank, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G=4096; R=[G*i//world for i in range(world+1)]
    full=torch.zeros((G,G)); send=full[R[rank]:R[rank+1]]
    pad=torch.zeros((G//world,G)); allf=torch.empty((G,G))
    for mode in ("dst","all","dst_sync"):
        dist.barrier(); t=time.perf_counter()
        for it in range(5):
            if mode=="all":
                dist.all_gather_into_tensor(allf, pad)
            else:
                if rank!=0: ops=[dist.P2POp(dist.isend, send, 0)]
                else: ops=[dist.P2POp(dist.irecv, full[R[r]:R[r+1]], r) for r in range(1,world)]
                ws=dist.batch_isend_irecv(ops)
                for w in ws: w.wait()
        dist.barrier()
        if rank==0: print(mode, (time.perf_counter()-t)/5*1e3, "ms")
    dist.destroy_process_group()
if __name__=="__main__":
    mp.spawn(run, args=(2,), nprocs=2)
