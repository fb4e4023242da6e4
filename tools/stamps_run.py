import os, sys
os.environ["BWRT_TUNING"] = "1"  # the library reads BWRT_* knobs only under it
sys.path[:0] = ["bwidman-raytracer_amd"]
import torch
from bwrt import Renderer, abi, scenes
key, W, H, SPP, MB, _ = scenes.CONFIGS[os.environ.get("CFG", "c3")]
lib = abi.load()
r = Renderer(0, lib=lib); r.set_scene(scenes.SCENES[key]())
for g in [int(x) for x in sys.argv[1:]]:
    img = torch.empty(-(-H // g) * W, dtype=torch.int32, device="cuda")
    p = r.params(W, H, SPP, MB, first_frame=1, row_offset=0, row_stride=g)
    r.init_rand(W, H, 0, g)
    os.environ.pop("BWRT_STAMPS", None)
    r.render_device(p, img.data_ptr(), None); torch.cuda.synchronize()
    os.environ["BWRT_STAMPS"] = "1"
    print("stride", g, flush=True)
    r.render_device(p, img.data_ptr(), None); torch.cuda.synchronize()
    os.environ.pop("BWRT_STAMPS", None)
