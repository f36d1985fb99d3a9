"""``jax.debug.visualize_array_sharding`` equivalent, rendered with rich.

Reference call sites: ``case1a.py:26,32,51``, ``case4_gspmd_ff.py:48,50,54``,
``case6_attention.py:164,198``.  One cell per shard block, labelled
``"<PLATFORM> <device ids>"`` (e.g. ``CPU 0,4``), coloured per device set.
Only rank <= 2 is supported (that is why the reference visualises ``x[0]``).
"""
from __future__ import annotations

import io
from typing import Optional

import rich.align
import rich.box
import rich.console
import rich.padding
import rich.style
import rich.table

from ..runtime.devices import get_device

__all__ = ["visualize_array_sharding", "visualize_sharding", "render_sharding_text"]

_PALETTE = [
    "#393b79", "#637939", "#8c6d31", "#843c39", "#7b4173", "#3182bd", "#31a354", "#756bb1",
    "#e6550d", "#636363", "#6baed6", "#74c476", "#9e9ac8", "#fd8d3c", "#969696", "#17becf",
]


def _blocks(shape, tile):
    """Return (nrows, ncols, {(i,j): device ids}, row sizes, col sizes) for a rank<=2 layout."""
    if len(shape) == 0:
        shape2, tiles = (1, 1), (1, 1)
        ids = {(0, 0): tile.holders(())}
    elif len(shape) == 1:
        shape2, tiles = (1, shape[0]), (1, tile.tile_shape[0])
        ids = {(0, j): tile.holders((j,)) for j in range(tiles[1])}
    elif len(shape) == 2:
        shape2, tiles = tuple(shape), tile.tile_shape
        ids = {(i, j): tile.holders((i, j)) for i in range(tiles[0]) for j in range(tiles[1])}
    else:
        raise ValueError(
            f"visualize_array_sharding only supports arrays of rank <= 2, got shape {tuple(shape)}")
    return shape2, tiles, ids


def visualize_sharding(shape, sharding, *, use_color: bool = True, scale: float = 1.0,
                       min_width: int = 9, max_width: int = 80, console=None):
    tile = sharding.tile_assignment(len(shape))
    (h, w), (tr, tc), ids = _blocks(tuple(shape), tile)
    base_height = max(1, int(10 * scale))
    aspect = w / h if h else 1.0
    total_w = max(min_width, min(max_width, int(base_height * aspect * 2.5 * scale)))
    total_h = max(1, min(base_height, int(total_w / aspect / 2.5) if aspect else base_height))
    cell_w = max(min_width, total_w // tc)
    cell_h = max(1, total_h // tr)

    table = rich.table.Table(show_header=False, show_lines=not use_color, padding=0,
                             highlight=not use_color, pad_edge=False,
                             box=rich.box.SQUARE if not use_color else None)
    color_of = {}
    for j in range(tc):
        table.add_column(width=cell_w, no_wrap=True)
    for i in range(tr):
        row = []
        for j in range(tc):
            devs = sorted(ids[(i, j)])
            platform = get_device(devs[0]).label
            label = f"{platform} " + ",".join(str(d) for d in devs)
            key = tuple(devs)
            if key not in color_of:
                color_of[key] = _PALETTE[len(color_of) % len(_PALETTE)]
            top = (cell_h - 1) // 2
            bottom = cell_h - 1 - top
            left = max(0, (cell_w - len(label)) // 2)
            right = max(0, cell_w - len(label) - left)
            style = rich.style.Style(color="white", bgcolor=color_of[key]) if use_color else None
            row.append(rich.padding.Padding(rich.align.Align(label, "center", vertical="middle"),
                                            (top, right, bottom, left), style=style))
        table.add_row(*row)
    console = console or rich.console.Console()
    console.print(table)


def visualize_array_sharding(arr, **kwargs):
    return visualize_sharding(arr.shape, arr.sharding, **kwargs)


def render_sharding_text(shape, sharding, **kwargs) -> str:
    """The plain-text (no colour) rendering, for golden tests."""
    buf = io.StringIO()
    con = rich.console.Console(file=buf, force_terminal=False, color_system=None, width=200)
    kwargs.setdefault("use_color", False)
    visualize_sharding(shape, sharding, console=con, **kwargs)
    return buf.getvalue()
