import torch, ctypes as C, sys
sys.path.insert(0, '/root/repo')
from rrin_amd import Net, _lib
from rrin_amd.engine import t_coefficients
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch
sd = keyed_state_dict(Net().state_dict())
net = Net(); net.load_state_dict(sd, strict=True); net = net.cuda().eval()
eng = net.engine()
lib = _lib.lib()
for n in (1, 2):
    i0, i1 = synthetic_batch(n, 64, 96, first_index=0); i0, i1 = i0.cuda(), i1.cuda()
    h, w = 64, 96
    outs = {}
    for use_scratch in (False, True):
        ws = torch.zeros(lib.rrin_net_workspace_bytes(n, h, w, eng.prec), dtype=torch.uint8, device="cuda")
        coef = t_coefficients(0.5, n).cuda()
        out = torch.empty_like(i0)
        d = _lib.NetDesc(n=n, h=h, w=w, i0=i0.data_ptr(), i1=i1.data_ptr(), out=out.data_ptr(), coef=coef.data_ptr(),
                         convs=eng.conv_table_for(n, h, w), heads=eng.head_table, workspace=ws.data_ptr(),
                         workspace_bytes=ws.numel(), prec=eng.prec)
        sc = None
        if use_scratch:
            nb = lib.rrin_net_scratch_bytes(C.byref(d)); print("scratch bytes", n, nb)
            sc = torch.zeros(max(nb, 1), dtype=torch.uint8, device="cuda")
            d.scratch, d.scratch_bytes = sc.data_ptr(), nb
        _lib.check(lib.rrin_net_fwd(C.byref(d), C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        outs[use_scratch] = out.clone()
    with torch.no_grad():
        ref1 = eng.forward(i0, i1, 0.5, streams=1)
        ref2 = net(i0, i1, 0.5)
    print(n, "noscratch vs scratch", (outs[False]-outs[True]).abs().max().item(),
          "scratch vs eng s1", (outs[True]-ref1).abs().max().item(), "eng s1 vs net", (ref1-ref2).abs().max().item())
