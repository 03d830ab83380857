"""Seeded synthetic KITTI-like RGB-D driving sequences.

A camera drives down a straight street: textured ground plane, two textured building walls,
sky, and optionally `n_objects` textured boxes ("cars") that move on their own trajectories.
Every pixel is ray-cast analytically, so depth, forward optical flow (frame t -> t+1) and the
semantic label map are exact and mutually consistent -- the inputs System::TrackRGBD expects:

  bgr   u8  [F, H, W, 3]   BGR image (memory order of the reference's cv::imread)
  disp  i16 [F, H, W]      disparity * 256 as uint16 bits (KITTI PNG convention, rgbd_tum.cc:127)
  flow  f32 [F, H, W, 2]   forward flow, pixels (the .flo fields, rgbd_tum.cc:131)
  mask  i32 [F, H, W]      semantic labels, 0 = static, 1..n_objects = boxes (LoadMask)

plus the ground-truth camera poses Tcw[F] and object poses Two[F, n_objects].

Generation runs with torch on the given device (GPU for the bench: frames are produced straight
into HBM before the timed region).  This is test/bench data plumbing, not part of the product.
"""
import math

import numpy as np
import torch

KITTI03 = dict(fx=721.5377, fy=721.5377, cx=609.5593, cy=172.8540, bf=387.5744)
CAM_HEIGHT = 1.65           # camera above the road (KITTI rig)
WALL_L, WALL_R = -7.0, 8.0  # building facades (world x)
WALL_TOP = -7.0             # facade top (world y, y points down)
BOX_HALF = (0.9, 0.75, 2.0)  # half extents of a car-sized box (x, y, z)


def _rot_y(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _se3(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


class StreetScene:
    """Trajectories of the camera and the objects (closed form in the frame index)."""

    def __init__(self, n_objects=3, seed=1003, speed=1.0, lanes=None):
        rng = np.random.default_rng(seed)
        self.seed = int(seed)
        self.speed = speed
        self.sway = (0.25 + 0.1 * rng.random(), 0.04 + 0.02 * rng.random())
        self.yaw = (0.02 + 0.01 * rng.random(), 0.03 + 0.01 * rng.random())
        lanes = lanes or [(-3.0, 12.0), (3.2, 16.0), (-0.3, 21.0), (3.4, 9.0), (-3.4, 19.0),
                          (0.0, 11.0), (-5.0, 14.0), (5.2, 20.0)]
        self.objs = []
        for k in range(n_objects):
            x0, d0 = lanes[k % len(lanes)]
            self.objs.append(dict(x0=x0, d0=d0, A=2.5 + rng.random(), w=0.04 + 0.02 * rng.random(),
                                  ph=2 * math.pi * rng.random(), lat=0.3 * rng.random(),
                                  yaw=0.05 * rng.random()))

    def Twc(self, t):
        x = self.sway[0] * math.sin(self.sway[1] * t)
        R = _rot_y(self.yaw[0] * math.sin(self.yaw[1] * t))
        return _se3(R, [x, 0.0, self.speed * t])

    def Two(self, k, t):
        o = self.objs[k]
        z = self.speed * t + o["d0"] + o["A"] * math.sin(o["w"] * t + o["ph"])
        x = o["x0"] + o["lat"] * math.sin(0.5 * o["w"] * t)
        R = _rot_y(o["yaw"] * math.sin(o["w"] * t))
        return _se3(R, [x, CAM_HEIGHT - BOX_HALF[1], z])


def _hash(ix, iy, salt):
    h = (ix * 374761393 + iy * 668265263 + salt * 1442695041) & 0xFFFFFFFF
    h = ((h ^ (h >> 13)) * 1274126177) & 0xFFFFFFFF
    h = h ^ (h >> 16)
    return (h & 0xFFFFFF).to(torch.float32) * (1.0 / 16777216.0)


def _vnoise(x, y, salt):
    x0 = torch.floor(x)
    y0 = torch.floor(y)
    fx = x - x0
    fy = y - y0
    fx = fx * fx * (3 - 2 * fx)
    fy = fy * fy * (3 - 2 * fy)
    ix = x0.to(torch.int64)
    iy = y0.to(torch.int64)
    a = _hash(ix, iy, salt)
    b = _hash(ix + 1, iy, salt)
    c = _hash(ix, iy + 1, salt)
    d = _hash(ix + 1, iy + 1, salt)
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def _texture(s, t, salt):
    """fbm + hard-edged blobs in surface coordinates (metres): corner-rich at every range."""
    acc = torch.zeros_like(s)
    amp, freq, norm = 1.0, 0.7, 0.0
    for o in range(6):
        acc = acc + amp * _vnoise(s * freq, t * freq, salt + 17 * o)
        norm += amp
        amp *= 0.6
        freq *= 2.0
    acc = acc / norm
    blobs = (_vnoise(s * 3.1, t * 3.1, salt + 999) > 0.55).to(torch.float32)
    return torch.clamp(30 + 150 * acc + 60 * blobs, 0, 255)


class SequenceRenderer:
    def __init__(self, scene, width=1242, height=375, K=KITTI03, device="cpu", aa=1):
        """aa > 1: the colour of a pixel is the mean of aa x aa sub-pixel rays (box-filtered
        texture, diagnostics of aliasing: tools/drift_ablation.py); depth, flow and labels stay
        the pixel centre's.  aa = 1 (default) is the sequence every test and the bench use."""
        self.scene, self.W, self.H, self.K = scene, width, height, K
        self.aa = int(aa)
        self.dev = torch.device(device)
        v, u = torch.meshgrid(torch.arange(height, dtype=torch.float64, device=self.dev),
                              torch.arange(width, dtype=torch.float64, device=self.dev),
                              indexing="ij")
        self.u, self.v = u, v
        self.ray = torch.stack([(u - K["cx"]) / K["fx"], (v - K["cy"]) / K["fy"],
                                torch.ones_like(u)], -1)  # camera ray with z = 1

    def _t(self, a):
        return torch.as_tensor(np.asarray(a), dtype=torch.float64, device=self.dev)

    def _cast(self, t, du=0.0, dv=0.0):
        """Depth Z (camera z), surface id, world hit point for frame t (rays through the pixel
        centres shifted by (du, dv) pixels)."""
        sc = self.scene
        Twc = self._t(sc.Twc(t))
        o = Twc[:3, 3]
        ray = self.ray
        if du or dv:
            ray = torch.stack([(self.u + du - self.K["cx"]) / self.K["fx"],
                               (self.v + dv - self.K["cy"]) / self.K["fy"],
                               torch.ones_like(self.u)], -1)
        dw = ray @ Twc[:3, :3].T  # world direction per unit camera depth
        inf = torch.full_like(self.u, float("inf"))
        Z = inf.clone()
        sid = torch.zeros_like(self.u, dtype=torch.int32)  # 0 sky
        dy, dx = dw[..., 1], dw[..., 0]
        zg = torch.where(dy > 1e-9, (CAM_HEIGHT - o[1]) / dy, inf)
        take = zg < Z
        Z = torch.where(take, zg, Z)
        sid = torch.where(take, torch.full_like(sid, 1), sid)
        for wall_x, code, sgn in ((WALL_L, 2, -1.0), (WALL_R, 3, 1.0)):
            zw = torch.where(sgn * dx > 1e-9, (wall_x - o[0]) / dx, inf)
            yw = o[1] + zw * dy
            zw = torch.where((yw > WALL_TOP) & (yw < CAM_HEIGHT), zw, inf)
            take = zw < Z
            Z = torch.where(take, zw, Z)
            sid = torch.where(take, torch.full_like(sid, code), sid)
        e = self._t(BOX_HALF)
        for k in range(len(sc.objs)):
            Two = self._t(sc.Two(k, t))
            Row = Two[:3, :3].T
            oo = Row @ (o - Two[:3, 3])
            do = dw @ Row.T
            with torch.no_grad():
                inv = 1.0 / torch.where(do.abs() < 1e-12, torch.full_like(do, 1e-12), do)
                t1 = (-e - oo) * inv
                t2 = (e - oo) * inv
                tn = torch.minimum(t1, t2).amax(-1)
                tf = torch.maximum(t1, t2).amin(-1)
            zb = torch.where((tn <= tf) & (tn > 0.1), tn, inf)
            take = zb < Z
            Z = torch.where(take, zb, Z)
            sid = torch.where(take, torch.full_like(sid, 10 + k), sid)
        Pw = o + Z.unsqueeze(-1).clamp(max=1e6) * dw
        return Z, sid, Pw

    def _project(self, Tcw, P):
        pc = P @ Tcw[:3, :3].T + Tcw[:3, 3]
        z = pc[..., 2]
        return pc[..., 0] / z * self.K["fx"] + self.K["cx"], pc[..., 1] / z * self.K["fy"] + \
            self.K["cy"]

    def _colour(self, t, sid, Pw):
        """Gray texture value and tint of every pixel from its ray's surface and hit point."""
        sc = self.scene
        g = torch.full_like(self.u, 200.0, dtype=torch.float64).to(torch.float32)
        tint = torch.zeros(self.H, self.W, 3, dtype=torch.float32, device=self.dev)
        P32 = Pw.to(torch.float32)
        seed = sc.seed
        surfaces = [(1, P32[..., 0], P32[..., 2], seed * 7 + 1, (0.95, 1.0, 1.05)),
                    (2, P32[..., 2], P32[..., 1], seed * 7 + 2, (1.1, 1.0, 0.9)),
                    (3, P32[..., 2], P32[..., 1], seed * 7 + 3, (0.9, 1.0, 1.1))]
        for code, s, tt, salt, col in surfaces:
            m = sid == code
            tex = _texture(s, tt, salt)
            g = torch.where(m, tex, g)
            tint = torch.where(m.unsqueeze(-1), torch.tensor(col, device=self.dev), tint)
        for k in range(len(sc.objs)):
            m = sid == 10 + k
            if not bool(m.any()):
                continue
            Two = self._t(sc.Two(k, t))
            Pl = ((Pw - Two[:3, 3]) @ Two[:3, :3]).to(torch.float32)
            ax = (Pl / torch.tensor(BOX_HALF, device=self.dev)).abs().argmax(-1)
            s = torch.where(ax == 0, Pl[..., 2], Pl[..., 0])
            tt = torch.where(ax == 1, Pl[..., 2], Pl[..., 1])
            tex = _texture(s + 13.0 * k, tt, seed * 7 + 100 + k)
            g = torch.where(m, tex, g)
            col = (1.0 + 0.15 * math.sin(k), 1.0, 1.0 - 0.15 * math.cos(k))
            tint = torch.where(m.unsqueeze(-1), torch.tensor(col, device=self.dev), tint)
        sky = sid == 0
        tint = torch.where(sky.unsqueeze(-1), torch.tensor((1.05, 1.0, 0.95), device=self.dev),
                           tint)
        return g, tint

    def frame(self, t):
        sc = self.scene
        Z, sid, Pw = self._cast(t)
        # ---- colour
        if self.aa <= 1:
            g, tint = self._colour(t, sid, Pw)
            bgr = torch.clamp(g.unsqueeze(-1) * tint + 0.5, 0, 255).to(torch.uint8)
        else:
            acc = torch.zeros(self.H, self.W, 3, dtype=torch.float32, device=self.dev)
            offs = [(k + 0.5) / self.aa - 0.5 for k in range(self.aa)]
            for dv in offs:
                for du in offs:
                    _, sid_s, Pw_s = self._cast(t, du, dv)
                    g_s, tint_s = self._colour(t, sid_s, Pw_s)
                    acc = acc + g_s.unsqueeze(-1) * tint_s
            bgr = torch.clamp(acc / (self.aa * self.aa) + 0.5, 0, 255).to(torch.uint8)
        # ---- disparity (KITTI u16 = disp * 256), exact depth where finite
        valid = torch.isfinite(Z) & (Z > 0.1)
        dq = torch.where(valid, torch.round(256.0 * self.K["bf"] / Z.clamp(min=0.1)),
                         torch.zeros_like(Z))
        dq = torch.where(dq <= 65535, dq, torch.zeros_like(dq))
        disp = dq.to(torch.int32).to(torch.int16)  # uint16 bits
        # ---- forward flow t -> t+1 (static points with the camera, boxes with their motion)
        Pn = Pw.clone()
        for k in range(len(sc.objs)):
            m = sid == 10 + k
            if not bool(m.any()):
                continue
            T0 = self._t(sc.Two(k, t))
            T1 = self._t(sc.Two(k, t + 1))
            Pl = (Pw - T0[:3, 3]) @ T0[:3, :3]
            Pn = torch.where(m.unsqueeze(-1), Pl @ T1[:3, :3].T + T1[:3, 3], Pn)
        Tcw1 = self._t(np.linalg.inv(sc.Twc(t + 1)))
        u1, v1 = self._project(Tcw1, Pn)
        fu = torch.where(valid, u1 - self.u, torch.zeros_like(u1))
        fv = torch.where(valid, v1 - self.v, torch.zeros_like(v1))
        flow = torch.stack([fu, fv], -1).to(torch.float32)
        mask = torch.where(sid >= 10, sid - 9, torch.zeros_like(sid)).to(torch.int32)
        return bgr, disp, flow, mask

    def sequence(self, nframes, start=0):
        F, H, W = nframes, self.H, self.W
        out = dict(bgr=torch.empty(F, H, W, 3, dtype=torch.uint8, device=self.dev),
                   disp=torch.empty(F, H, W, dtype=torch.int16, device=self.dev),
                   flow=torch.empty(F, H, W, 2, dtype=torch.float32, device=self.dev),
                   mask=torch.empty(F, H, W, dtype=torch.int32, device=self.dev))
        for i in range(F):
            b, d, f, m = self.frame(start + i)
            out["bgr"][i], out["disp"][i], out["flow"][i], out["mask"][i] = b, d, f, m
        out["Tcw"] = np.stack([np.linalg.inv(self.scene.Twc(start + i)) for i in range(F)])
        return out


def kitti_like_sequence(nframes, width=1242, height=375, n_objects=3, seed=1003, device="cpu",
                        start=0, lanes=None, aa=1):
    """C2 (n_objects=0) / C3 (n_objects=3) / C5 (1920x1080, n_objects=8) sequences; `lanes`
    (x, distance ahead) per object overrides the default street layout."""
    return SequenceRenderer(StreetScene(n_objects, seed, lanes=lanes), width, height,
                            device=device, aa=aa).sequence(nframes, start)


def to_numpy_frames(seq):
    """Host copies in the layout mmt_track_rgbd / oracle.Tracker.track take."""
    out = []
    for i in range(seq["bgr"].shape[0]):
        out.append(dict(bgr=seq["bgr"][i].cpu().numpy(),
                        disp=seq["disp"][i].cpu().numpy().view(np.uint16),
                        flow=seq["flow"][i].cpu().numpy(), sem=seq["mask"][i].cpu().numpy()))
    return out


def split_label_bands(mask, parts):
    """Each box label (1..3) split into `parts` rigid column bands with labels of their own
    (1 + (L - 1) parts + band), per frame, on the mask's device: BASELINE C5's eight rigid motions
    from two boxes (parts = 4).  Same bands as tests/test_gpu_track.py's split_labels."""
    import torch
    out = torch.zeros_like(mask)
    W = mask.shape[-1]
    cols = torch.arange(W, device=mask.device)
    for f in range(mask.shape[0]):
        o = out[f]
        for L in (1, 2, 3):
            m = mask[f] == L
            anyc = m.any(0).nonzero()
            if anyc.numel() == 0:
                continue
            u0 = int(anyc.min())
            w = int(anyc.max()) - u0 + 1
            q = torch.clamp(torch.div((cols - u0) * parts, w, rounding_mode="floor"), max=parts - 1)
            o[:] = torch.where(m, (1 + (L - 1) * parts + q)[None, :].to(mask.dtype), o)
    return out
