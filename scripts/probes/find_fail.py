import json, sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch, libiqo_amd, oracle_lib as ol
g = json.load(open('tests/golden/golden.json'))
bad = 0
for c in g['cases']:
    sw, sh, dw, dh = c['srcW'], c['srcH'], c['dstW'], c['dstH']
    if sw * sh > 4_000_000: continue
    r = libiqo_amd.make_resizer(c['method'], c['degree'], sw, sh, dw, dh, c['pxScale'])
    src = ol.gen(c['gen'], sw, sh, c['seed'])
    out = np.zeros((dh, dw), np.uint8)
    try:
        r.resize(sw, src, dw, out)
    except Exception as e:
        bad += 1
        if bad < 12:
            print(c['method'], c['degree'], sw, sh, dw, dh, c['pxScale'], r.describe()['kernel'], libiqo_amd.host_kernel_for(c['method'], c['degree'], sw, sh, dw, dh, c['pxScale']), e, flush=True)
print('failures', bad)
