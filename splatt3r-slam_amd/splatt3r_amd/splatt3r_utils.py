"""Inference / matching / rendering entry points of the SLAM frontend with the
reference's names and contracts (splatt3r_slam/splatt3r_utils.py).

Differences in HOW, not WHAT:
  * `decoder()` runs the fused pair plan (grouped decoder branches + both
    heads, HIP-graph replay) instead of `_decoder` + 2 x `_downstream_head`;
    the result dicts carry the same keys/shapes (:92-99).
  * `splatt3r_render()` feeds `render.pack_splats` (one HIP kernel for
    build_covariance + RGB2SH residual + scale-invariant rescale + triu)
    into the HIP rasterizer, instead of ~20 torch ops + render_cuda; same
    camera math (:332-432 -> decoder_splatting_cuda.py:30-83).
  * `gaussians_to_world()` is one HIP pass per view (include/s3w.h:
    strided gather, torch.quantile-exact depth bound, filters, stable
    compaction, world transform) instead of ~40 torch ops (:180-328).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

import lietorch
from splatt3r_amd import _lib, matching
from splatt3r_amd.config import config
from splatt3r_amd.render import (DecoderSplattingCUDA, camera_settings, camera_settings_sim3,
                                  normalize_intrinsics,
                                 pack_splats)

C0 = 0.28209479177387814


# ----------------------------------------------------------------- model ---
class Splatt3RModel:
    """What load_splatt3r returns (MAST3RGaussians, splatt3r_core/main.py:44-124):
    `.encoder` exposes _encode_image/_decoder/_downstream_head, `.decoder`
    is the splatting decoder."""

    def __init__(self, encoder, decoder):
        self.encoder = encoder
        self.decoder = decoder

    def eval(self):
        return self

    def share_memory(self):
        return self

    def to(self, *a, **k):
        return self


def load_splatt3r(path=None, device="cuda", cfg=None, seed: int = 1234, graphs: bool = True,
                  symmetric: bool = False):
    """splatt3r_utils.py:31-66.  `path`: a local Lightning ckpt / safetensors
    with the reference's state_dict keys (loaded with weights_only=True).  No
    path and no local checkpoints/epoch=19-step=1200.ckpt -> portable-PRNG
    weights of the same architecture (there is no download path offline)."""
    from splatt3r_amd.net import Splatt3RNet
    from splatt3r_amd.weights import FULL, load_state_dict_file
    cfg = cfg or FULL
    sd = None
    if path is None:
        local = os.path.join(os.getcwd(), "checkpoints", "epoch=19-step=1200.ckpt")
        path = local if os.path.exists(local) else None
    if path is not None:
        print(f"Loading Splatt3R model from {path}")
        sd = load_state_dict_file(path, device)
    net = Splatt3RNet(cfg, state_dict=sd, seed=seed, device=device, graphs=graphs,
                      symmetric=symmetric)
    return Splatt3RModel(net, DecoderSplattingCUDA([0.0, 0.0, 0.0]).to(device))


def load_retriever(splatt3r_model, retriever_path=None, device="cuda"):
    """splatt3r_utils.py:69-89: the keyframe retrieval database over the
    SLAM model's encoder, from the MASt3R retrieval checkpoint (default path
    as the reference) and the ASMK codebook beside it (.npy / .safetensors;
    retrieval_database.load_retrieval_weights)."""
    from splatt3r_amd.retrieval_database import RetrievalDatabase
    retriever_path = (
        "checkpoints/MASt3R_ViTLarge_BaseDecoder_512_catmlpdpt_metric_retrieval_trainingfree.pth"
        if retriever_path is None else retriever_path)
    return RetrievalDatabase(retriever_path, backbone=splatt3r_model.encoder, device=device)


# ------------------------------------------------------------- inference ---
@torch.inference_mode()
def decoder(model, feat1, feat2, pos1, pos2, shape1, shape2):
    """splatt3r_utils.py:92-99 (fused).  Returns (res1, res2) dicts of
    [B,H,W,...] tensors; they are views of the plan's static buffers and
    stay valid until the next decoder() call of the same shape."""
    H, W = _hw(shape1)
    res1, res2, _ = model.encoder.infer_pair(feat1, pos1, feat2, pos2, (H, W))
    return res1, res2


def _hw(shape):
    if torch.is_tensor(shape):
        s = shape.reshape(-1, 2)[0].tolist()
        return int(s[0]), int(s[1])
    s = np.asarray(shape).reshape(-1, 2)[0]
    return int(s[0]), int(s[1])


def downsample(X, C, D, Q):
    """splatt3r_utils.py:102-112."""
    ds = config["dataset"]["img_downsample"]
    if ds > 1:
        X = X[..., ::ds, ::ds, :].contiguous()
        C = C[..., ::ds, ::ds].contiguous()
        D = D[..., ::ds, ::ds, :].contiguous()
        Q = Q[..., ::ds, ::ds].contiguous()
    return X, C, D, Q


def _adjacent(a, b):
    return (a.dtype == b.dtype and a.shape == b.shape and a.is_contiguous() and
            b.is_contiguous() and
            a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr() and
            b.storage_offset() == a.storage_offset() + a.numel())


def _pair_view(a, b):
    """[2, *a.shape] over a and the adjacent b (no copy)."""
    return torch.empty(0, dtype=a.dtype, device=a.device).set_(
        a.untyped_storage(), a.storage_offset(), (2,) + tuple(a.shape))


def _clone_together(ts):
    """Fresh copies of the tensors `ts`.  When they tile one contiguous fp32
    range of a single storage (the pair plan's output blocks, net.py) that
    range is copied once and the copies are views into it; otherwise one
    clone each."""
    ts = list(ts)
    st = ts[0].untyped_storage()
    ok = all(t.dtype == torch.float32 and t.is_contiguous() and
             t.untyped_storage().data_ptr() == st.data_ptr() for t in ts)
    if ok:
        spans = sorted((t.storage_offset(), t.numel()) for t in ts)
        lo, hi = spans[0][0], spans[-1][0] + spans[-1][1]
        ok = all(a + n == b for (a, n), (b, _) in zip(spans, spans[1:]))
    if not ok:
        return [t.clone() for t in ts]
    copy = torch.empty(0, dtype=torch.float32, device=ts[0].device).set_(
        st, lo, (hi - lo,)).clone()
    return [copy[t.storage_offset() - lo:t.storage_offset() - lo + t.numel()].view(t.shape)
            for t in ts]


def _extract_gaussian_params(res):
    """splatt3r_utils.py:120-137 (copies: the plan buffers are reused)."""
    keys = ("means", "scales", "rotations", "sh", "opacities")
    d = dict(zip(keys, _clone_together(res[k] for k in keys)))
    if "conf" in res:
        d["conf"] = res["conf"].clone()
    return d


def _ensure_encoded(model, frame):
    if frame.feat is None:
        frame.feat, frame.pos, _ = model.encoder._encode_image(frame.img, frame.img_true_shape)


def _stack_outputs(res, clone=True):
    """torch.stack of the two heads' (pts3d, conf, desc, desc_conf) at batch
    element 0: one copy when the plan keeps them in one block (net.py), or
    (clone=False) views of that block, valid until the plan's next replay."""
    keys = ("pts3d", "conf", "desc", "desc_conf")
    r0, r1 = res
    if all(r0[k].shape[0] == 1 and _adjacent(r0[k], r1[k]) for k in keys):
        pv = [_pair_view(r0[k], r1[k]) for k in keys]
        X, C, D, Q = (t[:, 0] for t in (_clone_together(pv) if clone else pv))
        return downsample(X, C, D, Q)
    X = torch.stack([r["pts3d"][0] for r in res])
    C = torch.stack([r["conf"][0] for r in res])
    D = torch.stack([r["desc"][0] for r in res])
    Q = torch.stack([r["desc_conf"][0] for r in res])
    return downsample(X, C, D, Q)


@torch.inference_mode()
def splatt3r_inference_mono(model, frame):
    """splatt3r_utils.py:503-536."""
    _ensure_encoded(model, frame)
    res11, res21 = decoder(model, frame.feat, frame.feat, frame.pos, frame.pos,
                           frame.img_true_shape, frame.img_true_shape)
    frame.gaussian_pred = _extract_gaussian_params(res11)
    frame.gaussian_pred_cross = _extract_gaussian_params(res21)
    X, C, _, _ = _stack_outputs([res11, res21])
    Xii = X[0].reshape(1, -1, 3)
    Cii = C[0].reshape(1, -1, 1)
    return Xii[0], Cii[0]


def _slot(res, b):
    """Batch element b of a pair plan's result dict, as [1, ...] views."""
    return {k: v[b:b + 1] for k, v in res.items()}


def _ahead_key(frame, keyframe):
    return (frame.frame_id, keyframe.frame_id, keyframe.feat.data_ptr(),
            tuple(frame.img.shape))


def _decode_ahead(model, frame_i, frame_j, ahead):
    """Decoder + heads of (frame_i, frame_j), sharing one Bp = 2 pair-plan
    replay with the next frame (decode-ahead).

    The decoder of a tracked frame depends only on its encoder features and
    those of the last keyframe (splatt3r_utils.py:580-607), so the next
    frame's decode against the same keyframe can be issued with this one:
    one replay of the Bp = 2 plan (M = 1536-row GEMMs per branch) instead of
    two Bp = 1 replays.  Slot 1 is kept (views of the plan's output buffers,
    valid until the plan's next replay: `PairPlan.runs`) and used by the next
    call when that frame is tracked against the keyframe it was decoded
    against: the current keyframe, or frame_i when the predictor expects
    frame_i to be made the next keyframe; otherwise it is discarded.
    `ahead()` returns (next Frame -- encoded, its encoder ordered before the
    current stream --, the Frame to decode it against or None for frame_j)
    or None; it is only called when a decode is issued."""
    net = model.encoder
    cached = getattr(net, "_ahead_slot", None)
    net._ahead_slot = None
    if cached is not None:
        key, pp, runs = cached
        if key == _ahead_key(frame_i, frame_j) and pp.runs == runs:
            net.ahead_counts["used"] += 1
            return _slot(pp.res[0], 1), _slot(pp.res[1], 1), _desc16(pp, 1)
        net.ahead_counts["dropped"] += 1
    got = ahead() if ahead is not None else None
    nxt, against = got if got is not None else (None, None)
    # slot 1 decodes the next frame against the current keyframe (used when
    # frame_i stays a tracked frame) or against frame_i itself (used when
    # frame_i is made the next keyframe): the keyed keyframe must match
    against = frame_j if against is None else against
    if (nxt is None or nxt.feat is None or nxt.img.shape != frame_i.img.shape
            or nxt.feat.shape != frame_i.feat.shape or against.feat is None
            or against.feat.shape != frame_j.feat.shape):
        return _decode_alone(model, frame_i, frame_j)
    H, W = _hw(frame_i.img_true_shape)
    feat1 = torch.cat((frame_i.feat, nxt.feat))
    pos1 = torch.cat((frame_i.pos, nxt.pos))
    if against is frame_j:
        feat2, pos2 = frame_j.feat.expand(2, -1, -1), frame_j.pos.expand(2, -1, -1)
    else:
        feat2 = torch.cat((frame_j.feat, against.feat))
        pos2 = torch.cat((frame_j.pos, against.pos))
    r1, r2, pp = net.infer_pair(feat1, pos1, feat2, pos2, (H, W))
    net._ahead_slot = (_ahead_key(nxt, against), pp, pp.runs)
    net.ahead_counts["paired"] += 1
    return _slot(r1, 0), _slot(r2, 0), _desc16(pp, 0)


def _desc16(pp, b):
    """The pair plan's fp16 descriptor copies of pair b (net.py PairPlan.desc16,
    written by the Gaussian postprocess beside the fp32 desc) as [1, H, W, F]
    views of (head 1, head 2): the matching kernels' fp16 operands without a
    conversion pass; None when the plan has none."""
    d = getattr(pp, "desc16", None)
    return None if d is None else (d[0][b:b + 1], d[1][b:b + 1])


def _decode_alone(model, frame_i, frame_j):
    H, W = _hw(frame_i.img_true_shape)
    r1, r2, pp = model.encoder.infer_pair(frame_i.feat, frame_i.pos, frame_j.feat, frame_j.pos,
                                          (H, W))
    return r1, r2, _desc16(pp, 0)


def _tracker_decode(model, frame_i, frame_j, ahead=None):
    """(res_self, res_cross, desc16 pair or None) of the tracked pair."""
    _ensure_encoded(model, frame_i)
    _ensure_encoded(model, frame_j)
    if ahead is not None or getattr(model.encoder, "_ahead_slot", None) is not None:
        return _decode_ahead(model, frame_i, frame_j, ahead)
    return _decode_alone(model, frame_i, frame_j)


@torch.inference_mode()
def splatt3r_asymmetric_inference(model, frame_i, frame_j, ahead=None):
    """splatt3r_utils.py:580-607.  `ahead`: decode-ahead source of the next
    frame (see _decode_ahead); None decodes this pair alone."""
    res11, res21, _ = _tracker_decode(model, frame_i, frame_j, ahead)
    X, C, D, Q = _stack_outputs([res11, res21])
    return X, C, D, Q, (res11, res21)


def splatt3r_match_asymmetric(model, frame_i, frame_j, idx_i2j_init=None, ahead=None):
    """splatt3r_utils.py:610-644.

    The stacked (X, C, D, Q) the reference copies out (torch.stack) are
    views of the pair plan's output block here: every consumer reads them on
    the same stream before the plan's next replay (matching, the tracker's
    correspondence pass) or copies what it keeps (Frame.update_pointmap
    clones or fuses into new tensors), so the ~46 MB copy per tracked frame
    is not made.  Matching reads the plan's fp16 descriptors (the values
    .half() of the fp32 ones gives, written by the postprocess)."""
    res_self, res_cross, d16 = _tracker_decode(model, frame_i, frame_j, ahead)
    X, C, D, Q = _stack_outputs([res_self, res_cross], clone=False)
    frame_i.gaussian_pred = _extract_gaussian_params(res_self)
    frame_i.gaussian_pred_cross = _extract_gaussian_params(res_cross)
    b = X.shape[0] // 2
    if d16 is not None and X.shape[0] == 2 and config["dataset"]["img_downsample"] == 1:
        D1, D2 = d16
    else:
        D1, D2 = D[:b], D[b:]
    idx_i2j, valid_match_j = matching.match(X[:b], X[b:], D1, D2,
                                            idx_1_to_2_init=idx_i2j_init)
    Xii, Xji = X.reshape(2 * b, -1, 3)[:b], X.reshape(2 * b, -1, 3)[b:]
    Cii, Cji = C.reshape(2 * b, -1, 1)[:b], C.reshape(2 * b, -1, 1)[b:]
    Qii, Qji = Q.reshape(2 * b, -1, 1)[:b], Q.reshape(2 * b, -1, 1)[b:]
    # the reference unpacks the b=1 batch dim with einops (:638-641)
    return idx_i2j, valid_match_j, Xii[0], Cii[0], Qii[0], Xji[0], Cji[0], Qji[0]


@torch.inference_mode()
def splatt3r_decode_symmetric_batch(model, feat_i, pos_i, feat_j, pos_j, shape_i, shape_j,
                                    tag="backend"):
    """splatt3r_utils.py:466-499, batched: one fused pair plan over the b
    pairs in each order (the reference loops pairs one at a time).  The
    backend's plans (tag) are separate from the tracker's, so a backend
    worker thread can decode while the frontend tracks."""
    b = feat_i.shape[0]
    H, W = _hw(shape_i)
    r11, r21, _ = model.encoder.infer_pair(feat_i, pos_i, feat_j, pos_j, (H, W), tag=tag)
    keys = ("pts3d", "conf", "desc", "desc_conf")
    c11 = _clone_together([r11[k] for k in keys] + [r21[k] for k in keys])
    Xa, Ca, Da, Qa = ([c11[i], c11[4 + i]] for i in range(4))
    r22, r12, _ = model.encoder.infer_pair(feat_j, pos_j, feat_i, pos_i, (H, W), tag=tag)
    Xa += [r22["pts3d"], r12["pts3d"]]
    Ca += [r22["conf"], r12["conf"]]
    Da += [r22["desc"], r12["desc"]]
    Qa += [r22["desc_conf"], r12["desc_conf"]]
    # ordering 4 x b x h x w x c : [ii, ji, jj, ij]
    X, C, D, Q = (torch.stack(t, 0) for t in (Xa, Ca, Da, Qa))
    return downsample(X, C, D, Q)


def splatt3r_match_symmetric(model, feat_i, pos_i, feat_j, pos_j, shape_i, shape_j,
                             tag="backend"):
    """splatt3r_utils.py:539-576."""
    X, C, D, Q = splatt3r_decode_symmetric_batch(model, feat_i, pos_i, feat_j, pos_j,
                                                 shape_i, shape_j, tag)
    b = X.shape[1]
    Xii, Xji, Xjj, Xij = X
    Dii, Dji, Djj, Dij = D
    Qii, Qji, Qjj, Qij = Q
    idx, valid = matching.match(torch.cat((Xii, Xjj)), torch.cat((Xji, Xij)),
                                torch.cat((Dii, Djj)), torch.cat((Dji, Dij)))
    return (idx[:b], idx[b:], valid[:b], valid[b:], Qii.reshape(b, -1, 1),
            Qjj.reshape(b, -1, 1), Qji.reshape(b, -1, 1), Qij.reshape(b, -1, 1))


def splatt3r_match_directed(model, feat_a, pos_a, feat_b, pos_b, shape_a, shape_b,
                            tag="backend"):
    """One direction of splatt3r_match_symmetric (splatt3r_utils.py:539-576)
    for b ordered pairs (a, b): decode (a, b) once, match view a's own
    prediction against view b's prediction in a's frame.  Returns idx_a2b
    [b, hw], valid [b, hw, 1], Q_aa, Q_ba [b, hw, 1]: exactly the first half
    of the symmetric call's outputs for (a, b), or the second half for (b, a)
    -- so a pair's two directions can run on two ranks (pairs.PairShard).
    Every operation is per pair or per pixel, and the backend pair plans are
    batch-invariant, so the outputs do not depend on which pairs share a
    batch."""
    H, W = _hw(shape_a)
    r11, r21, _ = model.encoder.infer_pair(feat_a, pos_a, feat_b, pos_b, (H, W), tag=tag)
    X, C, D, Q = (torch.stack((r11[k], r21[k]), 0)
                  for k in ("pts3d", "conf", "desc", "desc_conf"))
    X, C, D, Q = downsample(X, C, D, Q)
    b = X.shape[1]
    idx, valid = matching.match(X[0].contiguous(), X[1].contiguous(), D[0].contiguous(),
                                D[1].contiguous())
    return idx, valid, Q[0].reshape(b, -1, 1).clone(), Q[1].reshape(b, -1, 1).clone()


# ------------------------------------------------------------- rendering ---
def _sim3_to_4x4(T_sim3):
    """splatt3r_utils.py:153-165: [sR | t; 0 0 0 1] (float32)."""
    data = T_sim3.data.detach()
    if data.dim() == 1:
        data = data.unsqueeze(0)
    return lietorch.Sim3(data.reshape(-1, 8)).matrix().to(torch.float32)


def _estimate_default_intrinsics(h, w, device="cuda"):
    """splatt3r_utils.py:168-176."""
    f = float(max(h, w))
    return torch.tensor([[f, 0, w / 2.0], [0, f, h / 2.0], [0, 0, 1]], device=device,
                        dtype=torch.float32)


class RasterSizing:
    """Binning capacity and depth-key width for the sync-free render
    (diff_gaussian_rasterization.rasterize_deferred), learnt from the frames
    already validated: capacity 1.25 x the most instances seen + 64k rounded
    up to a power of two (the binning buffer is then re-allocated only when
    the count crosses one, not whenever it sets a new maximum: a device
    allocation in the frame loop stalls the host), key width the widest seen
    + 1 bit.  Before the first validated frame the render takes the two-call
    path (one host read)."""

    def __init__(self):
        self.capacity = None
        self.key_bits = 32
        self.max_total = 0
        self.max_bits = 0
        self.rerenders = 0

    def update(self, total: int, bits=None):
        self.max_total = max(self.max_total, int(total))
        need = int(self.max_total * 1.25) + 65536
        self.capacity = 1 << (need - 1).bit_length()
        if bits is not None:
            self.max_bits = max(self.max_bits, int(bits))
            self.key_bits = min(32, self.max_bits + 1)


class RenderCheck:
    """The validity of a sync-free render: `info` (device int64[3] {status,
    instances, key bits}) and the two-call re-render to use when the frame
    did not fit.  Attached to the returned image as `_gsr_check`."""

    def __init__(self, info, rerender, sizing):
        self.info, self.rerender, self.sizing = info, rerender, sizing


@torch.inference_mode()
def splatt3r_render(model, frame, ref_frame, K=None, target_T_WC=None, sizing=None):
    """splatt3r_utils.py:332-432 -> [1,1,3,H,W].

    sizing (RasterSizing, the frame loop): render without a host read of
    the instance count (rasterize_deferred); the image then carries a
    RenderCheck (`image._gsr_check`) that its consumer resolves
    (Frontend._deliver) before using it."""
    if frame.gaussian_pred is None or frame.gaussian_pred_cross is None:
        print("[splatt3r_render] No Gaussian predictions available – skipping.")
        return None
    g1, g2 = frame.gaussian_pred, frame.gaussian_pred_cross
    dev = g1["means"].device
    _, h, w, _ = g1["means"].shape
    # intrinsics-only math on the host (cached), the pose part in one fp64
    # HIP thread: decoder_splatting_cuda.py:36-55 + cuda_splatting.py:67-113
    K_use = (_estimate_default_intrinsics(h, w, "cpu") if K is None
             else K.detach().to(device="cpu", dtype=torch.float32).clone())
    T_tgt = frame.T_WC if target_T_WC is None else target_T_WC
    bg = model.decoder.background_color.to(dev)
    settings, scale = camera_settings_sim3(frame.T_WC.data.to(dev), T_tgt.data.to(dev),
                                           K_use.reshape(-1, 3, 3)[0], (h, w), bg, near=0.1,
                                           far=1000.0, sh_degree=0)
    views = []
    for g, img in ((g1, frame.img), (g2, ref_frame.img)):
        views.append(dict(means=g["means"].reshape(-1, 3), scales=g["scales"].reshape(-1, 3),
                          rotations=g["rotations"].reshape(-1, 4), sh=g["sh"].reshape(-1, 3, 1),
                          opacities=g["opacities"].reshape(-1, 1),
                          img=img.to(dev)))
    means, cov6, shs, opac = pack_splats(views, float(scale[0]), img_chw_normalized=True)
    import diff_gaussian_rasterization as dgr
    rs = settings[0]

    def two_call():
        image, _ = dgr.GaussianRasterizer(rs)(means3D=means, means2D=torch.zeros_like(means),
                                              shs=shs, colors_precomp=None, opacities=opac,
                                              cov3D_precomp=cov6)
        return image[None, None]

    if sizing is None or sizing.capacity is None:
        out = two_call()
        if sizing is not None:
            sizing.update(dgr.last_num_rendered)
        return out
    image, _, info = dgr.rasterize_deferred(rs, means, opac, shs=shs, cov3D_precomp=cov6,
                                            capacity=sizing.capacity, key_bits=sizing.key_bits)
    out = image[None, None]
    out._gsr_check = RenderCheck(info, two_call, sizing)
    return out


class S3wView(ctypes.Structure):
    _fields_ = [("means", ctypes.c_void_p), ("scales", ctypes.c_void_p),
                ("rotations", ctypes.c_void_p), ("sh", ctypes.c_void_p),
                ("opacities", ctypes.c_void_p), ("conf", ctypes.c_void_p),
                ("img", ctypes.c_void_p), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("d_sh", ctypes.c_int), ("stride", ctypes.c_int)]


_P = ctypes.c_void_p
_lib.register({
    "s3w_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "s3w_set_path": (None, [ctypes.c_int]),
    "s3w_gaussians_to_world": (ctypes.c_int, [ctypes.POINTER(S3wView), _P, ctypes.c_float,
                                              ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                              _P, _P, _P, _P]),
})
_WS: dict = {}


def _workspace(dev, n):
    """The s3w scratch of the calling stream: one per (device, stream), so
    the frontend's world records (main or aux stream) and the backend
    worker's map refresh (its own stream) never share one concurrently."""
    need = _lib.lib().s3w_workspace_bytes(n)
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need:
        ws = _WS[key] = torch.empty(need, dtype=torch.uint8, device=dev)
    return ws


def world_records(view, img, T, stride=1, depth_min=float("-inf"), depth_max_percentile=1.0,
                  max_scale=float("inf"), min_confidence=0.0):
    """One predicted view ([H,W,...] tensors: means, scales, rotations, sh,
    opacities[, conf]) + its [3,H,W] ImgNorm image -> ([n,13] world records,
    device int64 count), stream-ordered (include/s3w.h).  T: device [4,4]
    (s R | t) float32.  Defaults disable every filter."""
    H, W, _ = view["means"].shape
    d_sh = view["sh"].shape[-1]
    n = -(-H // stride) * -(-W // stride)
    t = {k: view[k].float().contiguous() for k in
         ("means", "scales", "rotations", "sh", "opacities")}
    conf = view["conf"].float().contiguous() if view.get("conf") is not None else None
    im = img.float().contiguous()
    T = T.float().contiguous()
    _lib.require_cuda(*t.values(), im, T)
    v = S3wView(t["means"].data_ptr(), t["scales"].data_ptr(), t["rotations"].data_ptr(),
                t["sh"].data_ptr(), t["opacities"].data_ptr(),
                conf.data_ptr() if conf is not None else None, im.data_ptr(), H, W, d_sh, stride)
    out = torch.empty(n, 13, device=im.device)
    cnt = torch.empty(1, dtype=torch.int64, device=im.device)
    ws = _workspace(im.device, n)
    _lib.call("s3w_gaussians_to_world", ctypes.byref(v), T.data_ptr(), float(depth_min),
              float(depth_max_percentile), float(max_scale), float(min_confidence),
              ws.data_ptr(), out.data_ptr(), cnt.data_ptr(), _lib.stream(im.device))
    return out, cnt


@torch.inference_mode()
def gaussians_to_world(frame, include_cross=True, spatial_stride=1, depth_min=0.05,
                       depth_max_percentile=0.98, max_scale=0.5, min_confidence=1.5):
    """splatt3r_utils.py:180-328 -> (means_world [G,3], cov_triu [G,6],
    colors [G,3], opacities [G]); one HIP pass per view (include/s3w.h)
    and a single host sync for the record counts."""
    if frame.gaussian_pred is None:
        return None
    T = _sim3_to_4x4(frame.T_WC)[0].to(frame.img.device)
    preds = [frame.gaussian_pred]
    if include_cross and frame.gaussian_pred_cross is not None:
        preds.append(frame.gaussian_pred_cross)
    s = max(1, int(spatial_stride))
    img = frame.img
    outs, counts = [], []
    for pred in preds:
        for b in range(pred["means"].shape[0]):
            view = {k: v[b] for k, v in pred.items()}
            out, cnt = world_records(view, img[min(b, img.shape[0] - 1)], T, s, depth_min,
                                     depth_max_percentile, max_scale, min_confidence)
            outs.append(out)
            counts.append(cnt)
    counts = torch.cat(counts).tolist()
    recs = torch.cat([o[:c] for o, c in zip(outs, counts)]) if sum(counts) else None
    if recs is None:
        return None
    return (recs[:, 0:3].contiguous(), recs[:, 3:9].contiguous(), recs[:, 9:12].contiguous(),
            recs[:, 12].contiguous())


def _quat_to_matrix(q, eps: float = 1e-8):
    """utils/geometry.py:24-49 (xyzw, with the 2/(|q|^2+eps) factor)."""
    i, j, k, r = q.unbind(-1)
    two_s = 2 / ((q * q).sum(-1) + eps)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)),
                    -1)
    return o.reshape(*q.shape[:-1], 3, 3)


# ------------------------------------------------------------ host input ---
def resize_img(img, size, square_ok=False, return_transformation=False):
    """splatt3r_utils.py:658-693 (PIL resize + centre crop, ImgNorm)."""
    import PIL.Image
    assert size in (224, 512)
    pil = PIL.Image.fromarray(np.uint8(img * 255))
    W1, H1 = pil.size
    long_edge = round(size * max(W1 / H1, H1 / W1)) if size == 224 else size
    S = max(pil.size)
    interp = PIL.Image.LANCZOS if S > long_edge else PIL.Image.BICUBIC
    pil = pil.resize(tuple(int(round(x * long_edge / S)) for x in pil.size), interp)
    W, H = pil.size
    cx, cy = W // 2, H // 2
    if size == 224:
        half = min(cx, cy)
        pil = pil.crop((cx - half, cy - half, cx + half, cy + half))
    else:
        halfw, halfh = ((2 * cx) // 16) * 8, ((2 * cy) // 16) * 8
        if not square_ok and W == H:
            halfh = 3 * halfw / 4
        pil = pil.crop((cx - halfw, cy - halfh, cx + halfw, cy + halfh))
    arr = np.asarray(pil)
    t = torch.from_numpy(arr.astype(np.float32) / 255.0).permute(2, 0, 1)
    res = dict(img=((t - 0.5) / 0.5)[None], true_shape=np.int32([pil.size[::-1]]),
               unnormalized_img=arr)
    if return_transformation:
        return res, (W1 / W, H1 / H, (W - pil.size[0]) / 2, (H - pil.size[1]) / 2)
    return res
