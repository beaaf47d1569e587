"""Pure-Python restatement of the SPaRC-Gym step path.  TEST INFRASTRUCTURE ONLY.

One env over one puzzle dict (oracle pool format, see oracle/__init__.py).  Follows
/root/reference/SPaRC_Gym/SPaRC_Gym.py line by line (list-of-points path, np.clip legality,
O(S*L) solution compares, int/float reward types) so it doubles as the "reference-Python-speed"
CPU baseline in bench.py.  Pinned by tests/golden/*.json.gz.  Excludes the info-only
rule audit (_validate_rules, 941-950) and rendering.
"""
from __future__ import annotations

import numpy as np

# _action_to_direction, SPaRC_Gym.py:212-217
DIRS = {0: (1, 0), 1: (0, -1), 2: (-1, 0), 3: (0, 1)}


class CpuRefEnv:
    def __init__(self, puzzle, traceback=False, max_steps=2000):
        self.p = puzzle
        self.traceback = traceback
        self.max_steps = max_steps
        self.reset()

    # _load_puzzle state init (SPaRC_Gym.py:166-187), fresh planes
    def reset(self):
        p = self.p
        self.x_size, self.y_size = int(p["x_size"]), int(p["y_size"])
        self.gaps = np.asarray(p["gaps"])
        self.visited = np.zeros((self.x_size, self.y_size), np.int32)
        self.start = (int(p["start"][0]), int(p["start"][1]))
        self.target = (int(p["target"][0]), int(p["target"][1]))
        self.solution_paths = [[[int(a), int(b)] for a, b in s] for s in p["solution_paths"]]
        self.solution_count = int(p["solution_count"])
        self.path = [[self.start[0], self.start[1]]]
        self.loc = [self.start[0], self.start[1]]
        self.normal_reward = 0
        self.outcome_reward = 0
        self.current_step = 0
        self.visited[self.loc[0], self.loc[1]] = 1

    # _get_legal_actions (SPaRC_Gym.py:1024-1051)
    def legal_actions(self):
        legal = []
        for action, (dx, dy) in DIRS.items():
            nx, ny = self.loc[0] + dx, self.loc[1] + dy
            cx = min(max(nx, 0), self.x_size - 1)
            cy = min(max(ny, 0), self.y_size - 1)
            if self.gaps[cx, cy] == 0:
                if self.visited[cx, cy] == 1:
                    if self.traceback and len(self.path) >= 2:
                        if self.path[-2] == [cx, cy] and (nx, ny) == (cx, cy):
                            legal.append(action)
                elif (nx, ny) == (cx, cy):
                    legal.append(action)
        return legal

    @staticmethod
    def _on_solution_path(cur, sol):  # 1244-1265
        if len(cur) > len(sol):
            return False
        for i in range(len(cur)):
            if cur[i] != sol[i]:
                return False
        return True

    # step (SPaRC_Gym.py:1111-1238), returns (reward, terminated, truncated)
    def step(self, action):
        orig = list(self.loc)
        self.current_step += 1
        self.normal_reward = 0
        truncated = self.current_step >= self.max_steps
        if action in self.legal_actions():
            dx, dy = DIRS[action]
            nx, ny = self.loc[0] + dx, self.loc[1] + dy
            if self.visited[nx, ny] == 1:
                if self.traceback and self.path[-2] == [nx, ny]:
                    self.visited[self.loc[0], self.loc[1]] = 0
                    self.loc = [nx, ny]
                    self.visited[nx, ny] = 1
                    del self.path[-1]
            else:
                self.loc = [nx, ny]
                self.visited[nx, ny] = 1
                self.path.append([nx, ny])
        terminated = tuple(self.loc) == self.target
        if self.legal_actions() == []:
            truncated = True
        if terminated:
            truncated = False
        if terminated or truncated:
            for i in range(self.solution_count):
                if self.path == self.solution_paths[i]:
                    self.outcome_reward = 1
                    self.normal_reward = 1
                    break
            if self.outcome_reward != 1:
                self.outcome_reward = -1
                self.normal_reward = -1
        else:
            self.outcome_reward = 0
            if orig != self.loc:
                for i in range(self.solution_count):
                    if self._on_solution_path(self.path, self.solution_paths[i]):
                        self.normal_reward = 0.01
                        break
                    else:
                        self.normal_reward = -0.01
        return self.normal_reward, terminated, truncated
