import os, sys
sys.path.insert(0, "/root/repo")
from mitgcm_amd import configs
m = configs.make_model(configs.global_ocean_90x40x15)
os.environ["MGCM_NO_GRAPH"] = "1"
m.forward_step(4)
m.sync()
print("done")
