"""Physical constants (reference ``Source/Physics/PhysicsConst.h:7-14``)."""

import math

SPEED_OF_LIGHT = 2.99792458e8
EPS0 = 8.8541878176203892e-12
MU0 = 1.2566370614359173e-6
# relative convergence threshold of the amplitude (steady-state) mode
ACCURACY = 0.001
PI = math.pi
# free-space impedance
ETA0 = math.sqrt(MU0 / EPS0)
