"""open3d.visualization counterpart for headless runs.

The reference scripts end with an interactive window (check_one_frame.py:30, reconstruct_rgbd_gt.py:98,
hybrid_map.py:129).  Visualisation is out of scope and the GPU nodes have no display, so
draw_geometries validates its arguments and returns immediately — the scripts run to completion unchanged.
"""
from __future__ import annotations

import sys


def draw_geometries(geometry_list, window_name="Open3D", width=1920, height=1080, left=50, top=50,
                    point_show_normal=False, mesh_show_wireframe=False, mesh_show_back_face=False, **kwargs):
    """Open3D: blocks until the window closes.  Here: no window; reports what would have been shown."""
    items = list(geometry_list)
    print(f"[visualization] headless: {window_name!r} not displayed ({len(items)} geometries: "
          f"{', '.join(repr(g) for g in items)})", file=sys.stderr)
    return None
