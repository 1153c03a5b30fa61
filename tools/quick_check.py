import sys, time
sys.path.insert(0, '.')
import numpy as np, torch
print('cuda', torch.cuda.is_available(), torch.cuda.get_device_name(0))
from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
d = np.load('tests/golden/transfer_small.npz')
ws = [d[k] for k in sorted(k for k in d.files if k.startswith('w') and k[1:].isdigit())]
m, P = create_style_transfer_model((32,64,17),(32,64,3),8,8,1,weights=ws,max_batch=2)
y = m({'content': torch.from_numpy(d['content']).cuda(), 'style_params': torch.from_numpy(d['style_params']).cuda()})
torch.cuda.synchronize()
y = y.cpu().numpy()
print('small err', np.abs(y - d['output']).max())
