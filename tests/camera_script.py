"""A scripted interactive session for the progressive loop (src/main.cpp:600-718).

Each frame carries what InputHandler would hold (movement and rotation deltas,
the left mouse button, key events) and the frame time.  The script walks
through idle stretches (accumulation grows), WASD/space/shift movement, mouse
drags that wrap yaw past +-180 and clamp pitch at +-89, a held button with no
motion (reset without rotation), sub-threshold rotations whose length still
trips the reset, the R key (Camera::Reset + reset flag) and the L key (reset
flag only).  240 frames cross MoveAndRotate's 120-call re-orthonormalisation
twice.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class ScriptFrame:
    move: tuple
    rot: tuple
    mouse_left: bool
    key: str | None  # "R" (camera reset + flag), "L" (flag only) or None; handled before the frame
    dt: float


def camera_script(n: int = 240, seed: int = 2025) -> list[ScriptFrame]:
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        phase = (i // 12) % 8
        dt = float(np.float32(rng.uniform(0.004, 0.05)))
        move, rot, mouse, key = (0.0, 0.0, 0.0), (0.0, 0.0), False, None
        if phase == 1:    # keys: W/S/A/D/space/shift combinations
            move = tuple(float(x) for x in rng.integers(-1, 2, 3))
        elif phase == 2:  # mouse drag, large yaw steps wrap past +-180, pitch driven into the clamp
            mouse = True
            rot = (float(np.float32(rng.uniform(-45.0, 45.0))), float(np.float32(rng.uniform(-20.0, 30.0))))
        elif phase == 4:  # move while dragging
            mouse = True
            move = tuple(float(x) for x in rng.integers(-1, 2, 3))
            rot = (float(np.float32(rng.uniform(-5.0, 5.0))), float(np.float32(rng.uniform(-5.0, 5.0))))
        elif phase == 5:  # held button without motion, then tiny rotations (each |component| <= 1e-4)
            mouse = (i % 2 == 0)
            rot = (9e-5, 9e-5) if i % 3 == 0 else (0.0, 0.0)
        elif phase == 6:  # pitch held against -89
            mouse = True
            rot = (float(np.float32(rng.uniform(-2.0, 2.0))), -25.0)
        if i in (100, 190):
            key = "R"
        elif i in (60, 215):
            key = "L"
        out.append(ScriptFrame(move, rot, mouse, key, dt))
    return out
