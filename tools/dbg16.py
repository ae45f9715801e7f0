import numpy as np, torch, sys
sys.path.insert(0, "/root/repo")
from aimet_amd import _native, AimetTensorQuantizer
from aimet_amd.libpymo import TfEncoding, QuantizationMode
from aimet_amd.tensor_quantizer import IO_DTYPES
DEV="cuda"
for dtype in (torch.float16, torch.bfloat16):
    code = IO_DTYPES[dtype]
    e = TfEncoding(); e.min, e.max, e.bw = -0.001, 70000.0, 16
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF, num_channels=1)
    table = q.channelTable([e], torch.device(DEV))
    print("table", table.cpu().numpy().ravel().tolist())
    x = torch.arange(65536, dtype=torch.int32, device=DEV).to(torch.int16).view(dtype).contiguous()
    o16 = torch.empty_like(x)
    s = torch.cuda.current_stream().cuda_stream
    _native.call("aimet_qdq_per_channel_16", x.data_ptr(), o16.data_ptr(), 1, 1, 65536, code, table.data_ptr(), 0, 0, s)
    xf = x.float(); o32 = torch.empty_like(xf)
    _native.call("aimet_qdq_per_channel", xf.data_ptr(), o32.data_ptr(), 1, 1, 65536, table.data_ptr(), 0, 0, s)
    a = o16.view(torch.int16).cpu().numpy().astype(np.int64) & 0xffff
    b = o32.to(dtype).view(torch.int16).cpu().numpy().astype(np.int64) & 0xffff
    bad = np.nonzero(a != b)[0]
    print(dtype, "mismatches", len(bad))
    xs = xf.cpu().numpy()
    for i in list(bad[:12]) + list(bad[-6:]):
        print(hex(i), xs[i], hex(a[i]), hex(b[i]), o16[i].item(), o32[i].item())
