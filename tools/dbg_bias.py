import os, sys, socket
sys.path.insert(0, os.getcwd())
import numpy as np, torch, torch.distributed as dist, torch.multiprocessing as mp
from gasfm_amd import distributed as gd, synthetic

def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gasfm_amd
    from gasfm_amd import edge_block, _native
    from oracle.weights import deterministic_state_dict
    dev = torch.device("cuda", 0)
    sc = synthetic.scaled_config4(0.02, seed=5)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    model = gd.ShardedGraphAttnSfMNet(net.to(dev))
    data = gd.shard_scene(sc, rank, world, max_piece=64).to(dev)
    seen = []
    orig = edge_block.replicated_dbias
    def spy(g, defer):
        out = orig(g, defer)
        seen.append((tuple(g.shape), g.stride(), g.dtype, float(g.double().sum()), defer if isinstance(defer, bool) else len(defer), out))
        return out
    edge_block.replicated_dbias = spy
    g = torch.Generator().manual_seed(1)
    cP = torch.randn((sc.m, 3, 4), generator=g).to(dev)
    cX = torch.randn((4, sc.n), generator=g).to(dev)
    pred = model(data)
    loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX[:, data.point_slice]).sum()
    loss.backward()
    model.sync_grads()
    torch.cuda.synchronize()
    b0 = net.equivariant_blocks[0].global_feature_update.proj2view.graph_conv.bias
    msg = [f"rank {rank}: b0 bias grad {b0.grad.tolist()}"]
    for s in seen:
        msg.append(f"  spy g {s[0]} stride {s[1]} sum {s[3]:.5f} defer {s[4]} out {s[5].tolist()[:4]} same_as_b0grad {s[5].data_ptr()==b0.grad.data_ptr()}")
    q.put("\n".join(msg))
    dist.destroy_process_group()

if __name__ == "__main__":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn"); q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    for _ in ps: print(q.get(timeout=300))
    [p.join() for p in ps]
