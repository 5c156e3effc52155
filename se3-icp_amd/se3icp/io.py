"""Point-cloud file I/O used by the host side (PLY, the reference's only cloud format).

The reference reads clouds with ``open3d::io::CreatePointCloudFromFile`` /
``ReadPointCloud`` (examples/run_registration_method.cpp:27-31,
src/iterative_SE3_registration.cpp:350-370).  Only the vertex ``x y z``
properties matter for registration; every other element/property is skipped.
Supported encodings: ``ascii``, ``binary_little_endian`` and
``binary_big_endian``.  The C++ CLI has its own reader (csrc/ply.cpp) with the
same behaviour.
"""
from __future__ import annotations

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1",
    "short": "i2", "int16": "i2", "ushort": "u2", "uint16": "u2",
    "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


def _parse_header(f):
    line = f.readline().strip()
    if line != b"ply":
        raise ValueError("not a PLY file")
    fmt = None
    elements = []  # (name, count, [(prop_name, dtype | ('list', cnt_t, item_t))])
    while True:
        line = f.readline()
        if not line:
            raise ValueError("truncated PLY header")
        tok = line.decode("ascii", "replace").split()
        if not tok:
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append((tok[1], int(tok[2]), []))
        elif tok[0] == "property":
            if tok[1] == "list":
                elements[-1][2].append((tok[4], ("list", _PLY_TYPES[tok[2]], _PLY_TYPES[tok[3]])))
            else:
                elements[-1][2].append((tok[2], _PLY_TYPES[tok[1]]))
        elif tok[0] == "end_header":
            break
    return fmt, elements


def read_ply_xyz(path) -> np.ndarray:
    """Return the vertex positions of a PLY file as an (N, 3) float64 array."""
    with open(path, "rb") as f:
        fmt, elements = _parse_header(f)
        if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
            raise ValueError(f"unsupported PLY format {fmt!r}")
        endian = ">" if fmt == "binary_big_endian" else "<"
        for name, count, props in elements:
            if name == "vertex":
                names = [p[0] for p in props]
                for c in ("x", "y", "z"):
                    if c not in names:
                        raise ValueError("PLY vertex element lacks x/y/z")
                if any(isinstance(p[1], tuple) for p in props):
                    raise ValueError("list properties on vertices are not supported")
                if fmt == "ascii":
                    rows = [f.readline().split() for _ in range(count)]
                    arr = np.array(rows, dtype=np.float64).reshape(count, len(props))
                    cols = [names.index(c) for c in ("x", "y", "z")]
                    return np.ascontiguousarray(arr[:, cols])
                dt = np.dtype([(p[0], endian + p[1]) for p in props])
                data = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
                return np.stack([data["x"], data["y"], data["z"]], axis=1).astype(np.float64)
            # skip a non-vertex element that precedes the vertices
            if fmt == "ascii":
                for _ in range(count):
                    f.readline()
            else:
                if any(isinstance(p[1], tuple) for p in props):
                    raise ValueError("cannot skip a list element before the vertices")
                dt = np.dtype([(p[0], endian + p[1]) for p in props])
                f.read(dt.itemsize * count)
    raise ValueError("PLY file has no vertex element")


def write_ply_xyz(path, pts: np.ndarray, binary: bool = True) -> None:
    """Write an (N, 3) array as a PLY file with double x/y/z (Open3D's layout)."""
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    n = pts.shape[0]
    fmt = "binary_little_endian" if binary else "ascii"
    header = (f"ply\nformat {fmt} 1.0\ncomment se3icp\nelement vertex {n}\n"
              "property double x\nproperty double y\nproperty double z\nend_header\n")
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        if binary:
            f.write(pts.astype("<f8").tobytes())
        else:
            for p in pts:
                f.write(("%.17g %.17g %.17g\n" % tuple(p)).encode("ascii"))
