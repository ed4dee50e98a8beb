"""``python -m fdtd3d_amd [options]`` -- the fdtd3d command line driver."""

from .runner import main

main()
