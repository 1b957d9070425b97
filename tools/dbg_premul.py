import sys, os; sys.path.insert(0, os.getcwd())
import numpy as np, torch
import msccl_amd as M
os.environ.pop("MSCCL_XML_FILES", None)
for dt, tdt, val in [(8, torch.float64, 0.1), (7, torch.float32, 0.1), (4, torch.int64, 3)]:
    comms = M.Comm.init_all([0, 0])
    sb = np.array([val], dtype={8: np.float64, 7: np.float32, 4: np.int64}[dt]).tobytes()
    dev = torch.frombuffer(bytearray(sb), dtype=torch.uint8).cuda()
    ops = [c.create_premulsum(dev.data_ptr(), dt, 0) for c in comms]
    xs = [torch.full((1000,), 2, dtype=tdt, device="cuda") for _ in comms]
    torch.cuda.synchronize()
    with M.group():
        for c, x, o in zip(comms, xs, ops):
            c.all_reduce(x.data_ptr(), x.data_ptr(), 1000, dt, o, 0)
    torch.cuda.synchronize()
    print(dt, "device scalar:", xs[0][:4].tolist(), "expect", 2 * val * 2)
    for c in comms: c.destroy()
