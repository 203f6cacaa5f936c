import ctypes, os, torch
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdev_permlane.so"))
o = torch.zeros(384, dtype=torch.int32, device="cuda")
assert L.pl_run(ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
o = o.cpu().view(6, 64)
for n, r in zip(["16swap(x,x)[0]", "16swap(x,x)[1]", "32swap(x,x)[0]", "32swap(x,x)[1]", "16swap(x,x+100)[0]", "16swap(x,x+100)[1]"], o):
    print(n, r[[0, 1, 15, 16, 17, 31, 32, 33, 47, 48, 63]].tolist())
