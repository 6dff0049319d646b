import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # marl-maze_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
