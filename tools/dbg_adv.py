import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import wst_amd
from wst_amd import features
d = np.load("tests/golden/advstats.npz")
for name in ("rgb64_a", "rgb64_b", "struct64", "odd37x53", "gray128"):
    x = d[name + "_u8"].astype(np.float32) / 255.0
    got = features.extract_advanced_features_batch(x[None])[0].reshape(-1, 18)
    ref = d[name + "_ref"].reshape(-1, 18)
    for c in range(got.shape[0]):
        for k in [3, 4, 5, 9, 10, 11, 12, 13, 14, 17]:
            if got[c, k] != ref[c, k]:
                print(name, c, k, repr(got[c, k]), repr(ref[c, k]))
print("done")
