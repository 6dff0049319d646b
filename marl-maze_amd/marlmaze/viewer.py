"""Headless counterpart of the reference's pygame viewer (maze.py:276-522).

The reference draws the maze with pygame in a window and steps the policy on
key presses (``display_policy``: q reset, e one step, space run, s cycle the
view between the full maze and each agent's fogged view).  pygame and a
display are not part of this framework, so the same pictures are drawn into
images (PIL) instead, with the reference's geometry and colours:

* ``draw_maze(maze, id=-1)`` -- maze.py:277-301 (walls, marks, the shortest
  path's dots, start / end flags, agents with their eyes, the key), or for an
  agent tag maze.py:303-361 (``draw_hidden_maze``: fog except the cells along
  the agent's four rays up to ``vision_range`` and their side cells);
* ``display_policy(maze, id=-1, steps=..., path=...)`` -- maze.py:466-522's
  loop without the keyboard: reset, then ``steps`` policy steps (each agent's
  ``get_action`` on its observation, a reset after ``done``), one frame per
  state; the frames are returned and, with ``path``, saved as an animated GIF
  (``TIMESTEP_LENGTH`` per frame, as the reference's running mode).

``Maze.draw_maze`` / ``Maze.display_policy`` / ``Maze.print_maze`` call these.
"""
from PIL import Image, ImageColor, ImageDraw

CELL_SIZE = 40  # maze.py:12
AGENT_RADIUS = CELL_SIZE / 3
AGENT_EYE_RADIUS = AGENT_RADIUS / 3
TIMESTEP_LENGTH = 0.08  # maze.py:17
DELTAS = [(0, -1), (1, 0), (0, 1), (-1, 0)]  # maze.py:19

# pygame's named colours used by maze.py:6-10 and main.py:6-15 (X11 names with digits PIL does not know)
NAMED = {
    "white": (255, 255, 255), "black": (0, 0, 0), "mediumspringgreen": (0, 250, 154),
    "darkgoldenrod1": (255, 185, 15), "gray14": (36, 36, 36), "red": (255, 0, 0),
    "palevioletred1": (255, 130, 171), "royalblue1": (72, 118, 255), "darkslategray1": (151, 255, 255),
    "gold1": (255, 215, 0), "khaki1": (255, 246, 143),
}
PATH_COLOR = NAMED["white"]
WALL_COLOR = NAMED["black"]
FLAG_COLOR = NAMED["mediumspringgreen"]
KEY_COLOR = NAMED["darkgoldenrod1"]
FOG_COLOR = NAMED["gray14"]


def rgb(color):
    """An (r, g, b) tuple from a pygame.Color-like object (r, g, b attributes), a tuple / list, or a
    colour name (pygame's X11 names above, else PIL's)."""
    if hasattr(color, "r") and hasattr(color, "g") and hasattr(color, "b"):
        return (int(color.r), int(color.g), int(color.b))
    if isinstance(color, str):
        key = color.lower().replace(" ", "")
        return NAMED[key] if key in NAMED else ImageColor.getrgb(color)[:3]
    return tuple(int(v) for v in tuple(color)[:3])


class _Canvas:
    def __init__(self, maze, fill):
        self.img = Image.new("RGB", (maze.width * CELL_SIZE, maze.height * CELL_SIZE), fill)
        self.d = ImageDraw.Draw(self.img)

    def rect(self, color, x, y, w, h):  # pygame.draw.rect(screen, color, (x, y, w, h))
        self.d.rectangle([x, y, x + w - 1, y + h - 1], fill=color)

    def cell(self, color, x, y):
        self.rect(color, x * CELL_SIZE, y * CELL_SIZE, CELL_SIZE, CELL_SIZE)

    def circle(self, color, center, radius):
        cx, cy = center
        self.d.ellipse([cx - radius, cy - radius, cx + radius, cy + radius], fill=color)

    def polygon(self, color, points):
        self.d.polygon([tuple(p) for p in points], fill=color)


def cell_middle(x, y):  # maze.py:452-454
    return x * CELL_SIZE + CELL_SIZE // 2, y * CELL_SIZE + CELL_SIZE // 2


def _draw_one_agent(cv, agent, x, y, count, length):  # maze.py:371-404
    x, y = cell_middle(x, y)
    if length == 3:
        x, y = {0: (x - CELL_SIZE / 4, y - CELL_SIZE / 4), 1: (x + CELL_SIZE / 4, y - CELL_SIZE / 4),
                2: (x, y + CELL_SIZE / 4)}[count]
    elif length == 2:
        x = x - CELL_SIZE / 4 if count == 0 else x + CELL_SIZE / 4
    e = CELL_SIZE // 5
    eyes = {0: ((x + e, y - e), (x - e, y - e)), 1: ((x + e, y + e), (x + e, y - e)),
            2: ((x + e, y + e), (x - e, y + e)), 3: ((x - e, y + e), (x - e, y - e))}[agent.direction]
    if agent.has_key:
        cv.circle(KEY_COLOR, (x, y), CELL_SIZE / 2.3)
    cv.circle(rgb(agent.color), (x, y), AGENT_RADIUS)
    for c in eyes:
        cv.circle(WALL_COLOR, c, AGENT_EYE_RADIUS)


def _draw_agents(cv, maze):  # maze.py:363-369
    for (x, y), agents in maze.agent_positions.items():
        for count, agent in enumerate(agents):
            _draw_one_agent(cv, agent, x, y, count, len(agents))


def _draw_flags(cv, maze, start=True, end=True):  # maze.py:419-440
    flags = ([cell_middle(*maze.start)] if start else []) + ([cell_middle(*maze.end)] if end else [])
    for x, y in flags:
        rx, ry = x, y - CELL_SIZE / 1.2
        rw, rh = CELL_SIZE / 10, CELL_SIZE / 1.2
        tri = [(rx + rw, ry), (rx + rw, ry + rh // 2), (rx + rh // 2, (ry + ry + rh // 2) // 2)]
        cv.rect(WALL_COLOR, rx, ry, rw, rh)
        cv.polygon(FLAG_COLOR, tri)


def _draw_key(cv, maze):  # maze.py:442-450
    kx, ky = maze.key
    x, y = cell_middle(kx, ky)
    y -= CELL_SIZE / 4
    cv.circle(KEY_COLOR, (x, y), CELL_SIZE / 6)
    cv.circle(PATH_COLOR, (x, y), CELL_SIZE / 11)
    bx = kx * CELL_SIZE + CELL_SIZE / 2.2
    cv.rect(KEY_COLOR, bx, ky * CELL_SIZE + CELL_SIZE / 3, CELL_SIZE / 10, CELL_SIZE / 2)
    cv.rect(KEY_COLOR, bx, ky * CELL_SIZE + CELL_SIZE * 2 / 3, CELL_SIZE / 4.5, CELL_SIZE / 10)
    cv.rect(KEY_COLOR, bx, ky * CELL_SIZE + CELL_SIZE / 2, CELL_SIZE / 4.5, CELL_SIZE / 10)


def draw_maze(maze, id=-1):
    """The picture maze.py:277-301 draws (id = -1), or an agent's fogged view (id = its tag,
    maze.py:303-361).  Returns a PIL RGB image of width x height cells of CELL_SIZE pixels."""
    if id != -1:
        return draw_hidden_maze(maze, id)
    cv = _Canvas(maze, PATH_COLOR)
    layout = maze.layout
    tags = [a.tag for a in maze.agents]
    marks = [rgb(a.mark_color) for a in maze.agents]
    for y in range(maze.height):
        for x in range(maze.width):
            c = layout[y][x]
            if c == 1:
                cv.cell(WALL_COLOR, x, y)
            elif c in tags:
                cv.cell(marks[tags.index(c)], x, y)
    for x, y in maze.shortest_path or []:
        cv.circle(FLAG_COLOR, cell_middle(x, y), CELL_SIZE // 8)
    _draw_flags(cv, maze)
    _draw_agents(cv, maze)
    if maze.key != 0:
        _draw_key(cv, maze)
    return cv.img


def draw_hidden_maze(maze, agent_tag):
    """maze.py:303-361: fog, except the agent's cell and, per direction, the cells up to vision_range
    along the ray (stopping at a wall, which is drawn) and the two side cells of each."""
    agent = next((a for a in maze.agents if a.tag == agent_tag), None)
    other = next((a for a in maze.agents if a.tag != agent_tag), None)
    if agent is None:
        raise ValueError(f"no agent with tag {agent_tag}")
    cv = _Canvas(maze, FOG_COLOR)
    layout = maze.layout
    tags = [a.tag for a in maze.agents]
    marks = [rgb(a.mark_color) for a in maze.agents]
    key = end = start = False
    cv.cell(PATH_COLOR, agent.x, agent.y)
    for d, (dx, dy) in enumerate(DELTAS):
        nx, ny = agent.x, agent.y
        sx, sy = (1, 0) if d in (0, 2) else (0, 1)
        for _ in range(agent.vision_range):
            nx, ny = nx + dx, ny + dy
            if not maze.is_valid_cell(nx, ny):
                break
            if layout[ny][nx] == 1:
                cv.cell(WALL_COLOR, nx, ny)
                break
            key |= (nx, ny) == maze.key
            start |= (nx, ny) == maze.start
            end |= (nx, ny) == maze.end
            for k in (-1, 0, 1):
                x2, y2 = nx + sx * k, ny + sy * k
                if not maze.is_valid_cell(x2, y2):
                    continue
                c = layout[y2][x2]
                if c == 0:
                    cv.cell(PATH_COLOR, x2, y2)
                elif c == 1:
                    cv.cell(WALL_COLOR, x2, y2)
                elif c in tags:
                    cv.cell(marks[tags.index(c)], x2, y2)
                if (x2, y2) in maze.agent_positions and other is not None:
                    _draw_one_agent(cv, other, x2, y2, 0, 1)
    if key:
        _draw_key(cv, maze)
    if start or (agent.x, agent.y) == maze.start:
        _draw_flags(cv, maze, end=False)
    if agent.knows_end or end:
        _draw_flags(cv, maze, start=False)
    _draw_one_agent(cv, agent, agent.x, agent.y, 0, 1)
    return cv.img


def display_policy(maze, id=-1, steps=200, path=None):
    """maze.py:466-522 without the window: reset, then `steps` policy steps (a reset after done),
    one frame per state.  Returns the frames; with `path`, also writes them as an animated GIF."""
    obs, masks = maze.reset()
    frames = [draw_maze(maze, id)]
    for _ in range(int(steps)):
        action = [list(a.get_action(obs[i], masks[i])[0]) for i, a in enumerate(maze.agents)]
        obs, masks, _, done = maze.step(action)
        frames.append(draw_maze(maze, id))
        if done:
            obs, masks = maze.reset()
            frames.append(draw_maze(maze, id))
    if path is not None and frames:
        frames[0].save(path, save_all=True, append_images=frames[1:], duration=int(TIMESTEP_LENGTH * 1000),
                       loop=0)
    return frames
