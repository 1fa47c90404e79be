import torch, sys
sys.path.insert(0, '.')
import die_amd
from die_amd.ops import kernels as K
for (B,H,W) in [(1,37,45),(2,37,45),(1,224,224),(1,64,64),(1,37,32),(1,32,45)]:
    for split in (False, True):
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.zeros(B, H, W, 4, device="cuda")
        x[..., :3] = torch.rand(B, H, W, 3, device="cuda", generator=g) * 2 - 1
        w = torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 12.0
        bias = torch.randn(64, device="cuda", generator=g) * 0.1
        xin = x if split else x.to(torch.bfloat16)
        got = K.conv_stem7x7(xin, w, bias, relu=False, split=split).float()
        ref = torch.nn.functional.conv2d(xin[..., :3].float().permute(0, 3, 1, 2), w if split else w.bfloat16().float(), bias, stride=2, padding=3).permute(0,2,3,1)
        torch.cuda.synchronize()
        bad = ((got - ref).abs() > 1e-2 * (ref.abs() + 1)).any(-1)
        idx = bad.nonzero()
        print(B,H,W,'split' if split else 'bf16', 'bad pixels', int(bad.sum()), 'of', bad.numel(), idx[:3].tolist(), idx[-3:].tolist() if len(idx) else '')
