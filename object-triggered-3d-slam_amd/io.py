"""open3d.io counterparts: image read/write (PNG16 depth, JPEG/PNG colour) and binary PLY point clouds and
meshes.  File decode is host work in the reference too (reconstruct_rgbd_filter.py:91-93) and is outside the
timed hot path; arrays are uploaded to HBM by the first kernel that needs them.

PLY layout follows Open3D's writer: binary_little_endian, vertex x/y/z as double, nx/ny/nz double,
red/green/blue uchar (std::round(clip(c, 0, 1) * 255), half away from zero), faces as `list uchar int vertex_indices`.
"""
from __future__ import annotations

import os

import numpy as np

from .geometry import Image, PointCloud, TriangleMesh


def read_image(filename):
    """io.read_image: uint16 for 16-bit PNG depth (mm), uint8 HxWx3 RGB for colour, uint8 HxW for gray."""
    from PIL import Image as PILImage

    with PILImage.open(filename) as im:
        if im.mode in ("I;16", "I;16B", "I;16L", "I"):
            arr = np.array(im, dtype=np.uint16) if im.mode != "I" else np.array(im).astype(np.uint16)
        elif im.mode == "L":
            arr = np.array(im, dtype=np.uint8)
        else:
            arr = np.array(im.convert("RGB"), dtype=np.uint8)
    return Image(arr)


def write_image(filename, image, quality=-1):
    from PIL import Image as PILImage

    arr = np.asarray(image)
    if arr.dtype == np.uint16:
        PILImage.fromarray(arr).save(filename)
    else:
        kw = {"quality": int(quality)} if quality and quality > 0 else {}
        PILImage.fromarray(arr).save(filename, **kw)
    return True


# ------------------------------------------------------------------------------------------------ PLY
_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "<i2", "int16": "<i2",
              "ushort": "<u2", "uint16": "<u2", "int": "<i4", "int32": "<i4", "uint": "<u4", "uint32": "<u4",
              "float": "<f4", "float32": "<f4", "double": "<f8", "float64": "<f8"}


def _color_to_u8(c):
    """Open3D's utility::ColorToUint8 (written by write_point_cloud, reconstruct_rgbd_filter.py:140, and
    hybrid_map.py:121): uint8_t(std::round(std::min(1., std::max(0., c)) * 255.)).  std::max(0., NaN) is 0 and
    std::round rounds half AWAY from zero (np.round rounds half to even, which differs at k + 0.5).  x = v * 255 is
    one float64 rounding, as in C++; on [0, 255] x - floor(x) is exact, so the tie test is exact too."""
    c = np.asarray(c, np.float64)
    v = np.where(c > 0.0, c, 0.0)       # std::max(0., c): (0. < c) ? c : 0.
    v = np.where(v < 1.0, v, 1.0)       # std::min(1., v): (v < 1.) ? v : 1.
    x = v * 255.0
    f = np.floor(x)
    return (f + (x - f >= 0.5)).astype(np.uint8)


def _write_ply(filename, V, N=None, Cc=None, T=None):
    V = np.asarray(V, np.float64)
    fields = [("x", "<f8"), ("y", "<f8"), ("z", "<f8")]
    if N is not None:
        fields += [("nx", "<f8"), ("ny", "<f8"), ("nz", "<f8")]
    if Cc is not None:
        fields += [("red", "u1"), ("green", "u1"), ("blue", "u1")]
    rec = np.empty(V.shape[0], dtype=fields)
    rec["x"], rec["y"], rec["z"] = V[:, 0], V[:, 1], V[:, 2]
    if N is not None:
        N = np.asarray(N, np.float64)
        rec["nx"], rec["ny"], rec["nz"] = N[:, 0], N[:, 1], N[:, 2]
    if Cc is not None:
        c8 = _color_to_u8(np.asarray(Cc, np.float64))
        rec["red"], rec["green"], rec["blue"] = c8[:, 0], c8[:, 1], c8[:, 2]
    hdr = ["ply", "format binary_little_endian 1.0", "comment Created by otslam-mi355x",
           f"element vertex {V.shape[0]}"]
    names = {"<f8": "double", "u1": "uchar"}
    hdr += [f"property {names[t]} {n}" for n, t in fields]
    if T is not None:
        hdr += [f"element face {len(T)}", "property list uchar int vertex_indices"]
    hdr.append("end_header")
    d = os.path.dirname(os.path.abspath(filename))
    os.makedirs(d, exist_ok=True)
    with open(filename, "wb") as f:
        f.write(("\n".join(hdr) + "\n").encode("ascii"))
        f.write(rec.tobytes())
        if T is not None:
            T = np.asarray(T, np.int32)
            frec = np.empty(T.shape[0], dtype=[("n", "u1"), ("i", "<i4", (3,))])
            frec["n"] = 3
            frec["i"] = T
            f.write(frec.tobytes())
    return True


def _read_ply(filename):
    with open(filename, "rb") as f:
        if f.readline().strip() != b"ply":
            raise RuntimeError(f"[ReadPLY] {filename} is not a PLY file")
        fmt, elements = None, []
        while True:
            line = f.readline()
            if not line:
                raise RuntimeError(f"[ReadPLY] truncated header in {filename}")
            tok = line.decode("ascii", errors="replace").split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                elements.append([tok[1], int(tok[2]), []])
            elif tok[0] == "property":
                if tok[1] == "list":
                    elements[-1][2].append((tok[4], ("list", tok[2], tok[3])))
                else:
                    elements[-1][2].append((tok[2], tok[1]))
            elif tok[0] == "end_header":
                break
        out = {}
        if fmt == "ascii":
            rest = f.read().decode("ascii").split()
            pos = 0
            for name, count, props in elements:
                if any(isinstance(t, tuple) for _, t in props):
                    rows = []
                    for _ in range(count):
                        k = int(rest[pos])
                        rows.append([int(x) for x in rest[pos + 1:pos + 1 + k]])
                        pos += 1 + k
                    out[name] = {"vertex_indices": np.array(rows, np.int32)}
                else:
                    vals = np.array(rest[pos:pos + count * len(props)], dtype=np.float64).reshape(count, len(props))
                    pos += count * len(props)
                    out[name] = {p: vals[:, i] for i, (p, _) in enumerate(props)}
            return out
        if fmt != "binary_little_endian":
            raise RuntimeError(f"[ReadPLY] unsupported PLY format {fmt}")
        for name, count, props in elements:
            if any(isinstance(t, tuple) for _, t in props):
                (pname, (_, ct, it)), = [p for p in props if isinstance(p[1], tuple)]
                dt = np.dtype([("n", _PLY_TYPES[ct]), ("i", _PLY_TYPES[it], (3,))])
                raw = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
                if count and not np.all(raw["n"] == 3):
                    raise RuntimeError("[ReadPLY] only triangle faces are supported")
                out[name] = {pname: raw["i"].astype(np.int32)}
            else:
                dt = np.dtype([(p, _PLY_TYPES[t]) for p, t in props])
                raw = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
                out[name] = {p: raw[p] for p, _ in props}
        return out


def _stack(el, names, dtype=np.float64):
    if el is None or not all(n in el for n in names):
        return None
    return np.stack([np.asarray(el[n], dtype) for n in names], axis=1)


def _colors(el):
    c = _stack(el, ["red", "green", "blue"])
    if c is None:
        return None
    return c / 255.0


def read_point_cloud(filename, format="auto", remove_nan_points=False, remove_infinite_points=False,
                     print_progress=False):
    """io.read_point_cloud (hybrid_map.py:79).  Reads the vertex element of a PLY (a mesh PLY gives its
    vertices, as Open3D's PLY reader does)."""
    if not os.path.exists(filename):
        return PointCloud()
    data = _read_ply(filename)
    v = data.get("vertex")
    pcd = PointCloud()
    xyz = _stack(v, ["x", "y", "z"])
    if xyz is None:
        return pcd
    pcd.points = xyz
    c = _colors(v)
    if c is not None:
        pcd.colors = c
    n = _stack(v, ["nx", "ny", "nz"])
    if n is not None:
        pcd.normals = n
    return pcd


def write_point_cloud(filename, pointcloud, write_ascii=False, compressed=False, print_progress=False):
    """io.write_point_cloud (reconstruct_rgbd_filter.py:140, hybrid_map.py:121)."""
    V = np.asarray(pointcloud.points)
    N = np.asarray(pointcloud.normals) if pointcloud.has_normals() else None
    Cc = np.asarray(pointcloud.colors) if pointcloud.has_colors() else None
    return _write_ply(filename, V, N, Cc)


def read_triangle_mesh(filename, enable_post_processing=False, print_progress=False):
    if not os.path.exists(filename):
        return TriangleMesh()
    data = _read_ply(filename)
    v = data.get("vertex")
    f = data.get("face")
    V = _stack(v, ["x", "y", "z"])
    mesh = TriangleMesh()
    if V is None:
        return mesh
    mesh.vertices = V
    if f is not None and "vertex_indices" in f:
        mesh.triangles = f["vertex_indices"]
    c = _colors(v)
    if c is not None:
        mesh.vertex_colors = c
    n = _stack(v, ["nx", "ny", "nz"])
    if n is not None:
        mesh.vertex_normals = n
    return mesh


def write_triangle_mesh(filename, mesh, write_ascii=False, compressed=False, write_vertex_normals=True,
                        write_vertex_colors=True, write_triangle_uvs=True, print_progress=False):
    """io.write_triangle_mesh (reconstruct_rgbd.py:118)."""
    V = np.asarray(mesh.vertices)
    N = np.asarray(mesh.vertex_normals) if (write_vertex_normals and mesh.has_vertex_normals()) else None
    Cc = np.asarray(mesh.vertex_colors) if (write_vertex_colors and mesh.has_vertex_colors()) else None
    return _write_ply(filename, V, N, Cc, np.asarray(mesh.triangles))
