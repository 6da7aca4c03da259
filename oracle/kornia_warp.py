"""ORACLE / TEST INFRASTRUCTURE ONLY -- restatement of kornia 0.6.3 ``warp_perspective``.

Never imported by the product path (``deep-multiview-depth-estimation_amd/mvs_amd``); only by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.

Why it exists: the reference calls ``kornia.geometry.transform.warp_perspective`` at
``scripts/homography.py:86`` (kornia==0.6.3 pinned at ``requirements.txt:1``).  kornia is a
third-party dependency that is not vendored under /root/reference and is not installed here, so
its published algorithm is restated below, function by function, from kornia 0.6.3:

  * ``normal_transform_pixel``  (kornia/geometry/conversions.py)  pixel -> [-1, 1] map using the
    (size - 1) denominator, eps 1e-14 when size == 1;
  * ``normalize_homography``    (kornia/geometry/transform/imgwarp.py)
    ``dst_norm_T_src_norm = N_dst @ (M @ inv(N_src))``;
  * ``create_meshgrid``         (kornia/utils/grid.py) normalised: ``(linspace(0,W-1,W)/(W-1)-0.5)*2``;
  * ``convert_points_from_homogeneous`` (kornia/geometry/conversions.py, eps 1e-8):
    ``scale = 1/(z+eps)`` where ``|z| > eps`` else 1;
  * ``transform_points``        (kornia/geometry/linalg.py) ``bmm(points_h, T^T)`` then dehomogenise;
  * ``warp_perspective``        (kornia/geometry/transform/imgwarp.py) -> ``F.grid_sample`` with the
    caller's ``align_corners`` (the reference passes ``False``), bilinear, zero padding.

Parity status: **unpinned against real kornia** (not present in this container, no fixtures in the
reference hold its outputs).  It is pinned against analytic known answers in
``tests/test_oracle.py`` (identity-H law ``ix = x*w/(w-1) - 0.5``, pure translation, all
out-of-bounds, the ``|s| <= 1e-8`` branch).
"""
import torch
import torch.nn.functional as F


def normal_transform_pixel(height: int, width: int, eps: float = 1e-14,
                           device=None, dtype=torch.float32) -> torch.Tensor:
    den_w = eps if width == 1 else width - 1.0
    den_h = eps if height == 1 else height - 1.0
    m = torch.tensor([[1.0, 0.0, -1.0], [0.0, 1.0, -1.0], [0.0, 0.0, 1.0]],
                     device=device, dtype=dtype)
    m[0, 0] = m[0, 0] * 2.0 / den_w
    m[1, 1] = m[1, 1] * 2.0 / den_h
    return m.unsqueeze(0)


def normalize_homography(dst_pix_trans_src_pix: torch.Tensor, dsize_src, dsize_dst) -> torch.Tensor:
    src_h, src_w = dsize_src
    dst_h, dst_w = dsize_dst
    n_src = normal_transform_pixel(src_h, src_w).to(dst_pix_trans_src_pix)
    n_src_inv = torch.inverse(n_src)
    n_dst = normal_transform_pixel(dst_h, dst_w).to(dst_pix_trans_src_pix)
    return n_dst @ (dst_pix_trans_src_pix @ n_src_inv)


def create_meshgrid(height: int, width: int, device=None, dtype=torch.float32) -> torch.Tensor:
    xs = torch.linspace(0, width - 1, width, device=device, dtype=dtype)
    ys = torch.linspace(0, height - 1, height, device=device, dtype=dtype)
    xs = (xs / (width - 1) - 0.5) * 2
    ys = (ys / (height - 1) - 0.5) * 2
    gx, gy = torch.meshgrid(xs, ys, indexing="ij")
    grid = torch.stack((gx, gy)).transpose(1, 2)          # 2 x H x W
    return grid.unsqueeze(0).permute(0, 2, 3, 1)           # 1 x H x W x 2


def convert_points_from_homogeneous(points: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    z = points[..., -1:]
    keep = torch.abs(z) > eps
    scale = torch.where(keep, torch.tensor(1.0, dtype=points.dtype) / (z + eps), torch.ones_like(z))
    return scale * points[..., :-1]


def transform_points(trans_01: torch.Tensor, points_1: torch.Tensor) -> torch.Tensor:
    shape = list(points_1.shape)
    pts = points_1.reshape(-1, points_1.shape[-2], points_1.shape[-1])
    trans = trans_01.reshape(-1, trans_01.shape[-2], trans_01.shape[-1])
    trans = torch.repeat_interleave(trans, repeats=pts.shape[0] // trans.shape[0], dim=0)
    pts_h = torch.nn.functional.pad(pts, [0, 1], "constant", 1.0)
    out_h = torch.bmm(pts_h, trans.permute(0, 2, 1))
    out = convert_points_from_homogeneous(out_h)
    shape[-2] = out.shape[-2]
    shape[-1] = out.shape[-1]
    return out.reshape(shape)


def warp_perspective(src: torch.Tensor, M: torch.Tensor, dsize, mode: str = "bilinear",
                     padding_mode: str = "zeros", align_corners: bool = True) -> torch.Tensor:
    if src.dim() != 4:
        raise ValueError("src must be B x C x H x W, got %s" % (tuple(src.shape),))
    if M.dim() != 3 or M.shape[-2:] != (3, 3):
        raise ValueError("M must be B x 3 x 3, got %s" % (tuple(M.shape),))
    B, _, H, W = src.shape
    h_out, w_out = dsize
    dst_norm_T_src_norm = normalize_homography(M, (H, W), (h_out, w_out))
    src_norm_T_dst_norm = torch.inverse(dst_norm_T_src_norm)
    return warp_normalized(src, src_norm_T_dst_norm, dsize, mode, padding_mode, align_corners)


def warp_normalized(src: torch.Tensor, G: torch.Tensor, dsize, mode: str = "bilinear",
                    padding_mode: str = "zeros", align_corners: bool = True) -> torch.Tensor:
    """The second half of ``warp_perspective``: sample ``src`` through a GIVEN normalised sampling
    matrix ``G = src_norm_T_dst_norm`` (B x 3 x 3, src's dtype) -- kornia's meshgrid,
    ``transform_points`` and ``grid_sample`` exactly as above.  Lets a test hand the oracle the
    matrices the HIP kernels formed (fp64 algebra, stored fp32), isolating the sampling arithmetic
    from the reference's fp32 homography composition."""
    B = src.shape[0]
    h_out, w_out = dsize
    grid = create_meshgrid(h_out, w_out, device=src.device, dtype=src.dtype).repeat(B, 1, 1, 1)
    grid = transform_points(G[:, None, None], grid)
    return F.grid_sample(src, grid, mode=mode, padding_mode=padding_mode, align_corners=align_corners)
