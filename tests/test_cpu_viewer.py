"""The headless viewer (marlmaze/viewer.py, maze.py:276-522's pictures) on a
stub maze: no GPU, no pygame."""
import types

import numpy as np

from marlmaze import viewer


def _stub():
    layout = [[1, 1, 1, 1, 1],
              [1, 0, 2, 0, 1],
              [1, 0, 1, 3, 1],
              [1, 0, 0, 0, 1],
              [1, 1, 1, 1, 1]]
    a = types.SimpleNamespace(tag=2, color=(255, 0, 0), mark_color="palevioletred1", x=1, y=1, direction=2,
                              has_key=False, knows_end=False, vision_range=4)
    b = types.SimpleNamespace(tag=3, color="royalblue1", mark_color=(151, 255, 255), x=3, y=3, direction=0,
                              has_key=True, knows_end=True, vision_range=4)
    m = types.SimpleNamespace(width=5, height=5, layout=layout, agents=(a, b), shortest_path=[(1, 1), (1, 2)],
                              start=(1, 1), end=(3, 3), key=(1, 3), agent_positions={(1, 1): [a], (3, 3): [b]})
    m.is_valid_cell = lambda x, y: 0 <= x < 5 and 0 <= y < 5
    return m, a, b


def test_full_view_cells_and_agents():
    m, a, b = _stub()
    img = np.asarray(viewer.draw_maze(m))
    C = viewer.CELL_SIZE
    assert img.shape == (5 * C, 5 * C, 3)
    assert tuple(img[2, 2]) == viewer.WALL_COLOR                           # wall cell (0, 0)
    assert tuple(img[1 * C + 2, 2 * C + 2]) == viewer.rgb("palevioletred1")  # agent 2's mark at (2, 1)
    assert tuple(img[2 * C + 2, 3 * C + 2]) == (151, 255, 255)              # agent 3's mark at (3, 2)
    assert tuple(img[3 * C + 2, 2 * C + 2]) == viewer.PATH_COLOR            # open cell (2, 3)
    assert tuple(img[1 * C + C // 2 - 3, 1 * C + C // 2 + 8]) == (255, 0, 0)  # agent body
    # agent 3 holds the key: the key-coloured ring around its body
    assert tuple(img[3 * C + C // 2, 3 * C + C // 2 + 15]) == viewer.KEY_COLOR


def test_hidden_view_fog_and_rays():
    m, a, b = _stub()
    img = np.asarray(viewer.draw_maze(m, id=2))
    C = viewer.CELL_SIZE
    assert tuple(img[1 * C + 2, 1 * C + 2]) == viewer.PATH_COLOR    # own cell
    assert tuple(img[2 * C + 2, 1 * C + 2]) == viewer.PATH_COLOR    # down the ray (1, 2)
    assert tuple(img[2 * C + 2, 2 * C + 2]) == viewer.WALL_COLOR    # its side cell (2, 2): a wall
    assert tuple(img[1 * C + 2, 2 * C + 2]) == viewer.rgb("palevioletred1")  # right: the mark cell
    assert tuple(img[2 * C + 2, 3 * C + 2]) == (151, 255, 255)     # (3, 2): side cell of the right ray
    assert tuple(img[3 * C + 2, 3 * C + 2]) == viewer.FOG_COLOR     # (3, 3): on none of its rays
    assert tuple(img[3 * C + C // 2, 3 * C + C // 2]) == viewer.FOG_COLOR  # so the other agent is not drawn


def test_colour_names():
    assert viewer.rgb("royalblue1") == (72, 118, 255)
    assert viewer.rgb(types.SimpleNamespace(r=1, g=2, b=3, a=255)) == (1, 2, 3)
    assert viewer.rgb("white") == (255, 255, 255)
