"""Debug: HIP full-map render vs oracle on the viz golden (radii, pixels)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splatt3r-slam_amd")]
import oracle
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
g = np.load(os.path.join(REPO, "tests/golden/viz_render.npz"))
dev = "cuda"
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
for bg in (g["settings_bg"], np.zeros(3, np.float32)):
    st = GaussianRasterizationSettings(
        image_height=int(g["settings_image_height"]), image_width=int(g["settings_image_width"]),
        tanfovx=float(g["settings_tanfovx"]), tanfovy=float(g["settings_tanfovy"]), bg=t(bg),
        scale_modifier=1.0, viewmatrix=t(g["settings_viewmatrix"]), projmatrix=t(g["settings_projmatrix"]),
        sh_degree=0, campos=t(g["settings_campos"]), prefiltered=False, debug=False)
    m = t(g["in_means3D"])
    img, radii = GaussianRasterizer(st)(means3D=m, means2D=torch.zeros_like(m), shs=None,
                                        colors_precomp=t(g["colors"]), opacities=t(g["opacities"][:, None]),
                                        cov3D_precomp=t(g["in_cov3D_precomp"]))
    sd = dict(image_height=int(g["settings_image_height"]), image_width=int(g["settings_image_width"]),
              tanfovx=float(g["settings_tanfovx"]), tanfovy=float(g["settings_tanfovy"]), bg=bg,
              viewmatrix=g["settings_viewmatrix"], projmatrix=g["settings_projmatrix"], sh_degree=0,
              campos=g["settings_campos"])
    ref = oracle.raster(sd, g["in_means3D"], g["opacities"], colors_precomp=g["colors"],
                        cov3D_precomp=g["in_cov3D_precomp"])
    a = img.cpu().numpy(); r = radii.cpu().numpy()
    d = np.abs(a - ref["color"])
    print("bg", bg, "radii mismatches", int((r != ref["radii"]).sum()), "pixel mismatches",
          int((d > 0).sum()), "max", float(d.max()))
    ys, xs = np.nonzero(d.max(0) > 0)
    print("  first mismatching pixels (y, x):", list(zip(ys[:10].tolist(), xs[:10].tolist())))
    if bg.any():
        print("  golden vs oracle now:", float(np.abs(np.clip(ref["color"], 0, 1).transpose(1, 2, 0) - g["image_hwc"]).max()))

print("---- through the map")
from splatt3r_amd.gaussian_map import SharedGaussians, gl_to_cv_T_WC, render_map, viz_camera
gm = SharedGaussians(max_gaussians=1 << 16, device=dev)
gm.append(t(g["means"]), t(g["cov6"]), t(g["colors"]), t(g["opacities"]), kf_idx=0, opacity_threshold=0.0)
print("n", gm.n_gaussians, "means eq", bool((gm.means[:30000].cpu().numpy() == g["means"]).all()),
      "cov eq", bool((gm.cov_triu[:30000].cpu().numpy() == g["cov6"]).all()),
      "col eq", bool((gm.colors[:30000].cpu().numpy() == g["colors"]).all()),
      "op eq", bool((gm.opacities[:30000].cpu().numpy() == g["opacities"]).all()))
Twc = gl_to_cv_T_WC(g["T_CW_gl"])
for rep in range(3):
    img = render_map(gm, Twc, 320, 240, 45.0, clamp=False)
    a = img.cpu().numpy()
    ref = oracle.raster(dict(image_height=240, image_width=320, tanfovx=float(g["settings_tanfovx"]),
                             tanfovy=float(g["settings_tanfovy"]), bg=g["settings_bg"],
                             viewmatrix=g["settings_viewmatrix"], projmatrix=g["settings_projmatrix"],
                             sh_degree=0, campos=g["settings_campos"]),
                        g["in_means3D"], g["opacities"], colors_precomp=g["colors"],
                        cov3D_precomp=g["in_cov3D_precomp"])
    d = np.abs(a - ref["color"])
    print("rep", rep, "pixel mismatches", int((d > 0).sum()), "max", float(d.max()))
tx, ty, view_t, full_proj, campos, s, s2 = viz_camera(Twc, 320, 240, 45.0)
sc_means = torch.empty(30000, 3, device=dev); sc_cov = torch.empty(30000, 6, device=dev)
from splatt3r_amd import _lib
_lib.call("s3w_map_scale", gm.means.data_ptr(), gm.cov_triu.data_ptr(), gm._n.data_ptr(), 30000,
          float(s), float(s2), sc_means.data_ptr(), sc_cov.data_ptr(), _lib.stream())
print("scaled means eq", bool((sc_means.cpu().numpy() == g["in_means3D"]).all()),
      "scaled cov eq", bool((sc_cov.cpu().numpy() == g["in_cov3D_precomp"]).all()),
      float(np.abs(sc_cov.cpu().numpy() - g["in_cov3D_precomp"]).max()))
print("---- settings captured from render_map")
import diff_gaussian_rasterization as dgr
cap = {}
orig = dgr.GaussianRasterizer
import splatt3r_amd.gaussian_map as GMm
class Cap(orig):
    def __init__(self, rs):
        cap["rs"] = rs
        super().__init__(rs)
dgr.GaussianRasterizer = Cap
render_map(gm, Twc, 320, 240, 45.0, clamp=False)
rs = cap["rs"]
for k in ("tanfovx", "tanfovy", "image_height", "image_width", "sh_degree", "scale_modifier"):
    print(k, getattr(rs, k), g.get("settings_" + k) if ("settings_" + k) in g.files else None)
for k in ("bg", "viewmatrix", "projmatrix", "campos"):
    v = getattr(rs, k)
    v = v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)
    print(k, "maxdiff", float(np.abs(v.reshape(-1) - g["settings_" + k].reshape(-1)).max()), v.dtype)
