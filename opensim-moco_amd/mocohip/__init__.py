"""mocohip — MI355X-native Moco direct-collocation hot path (host side).

The product is libmocohip.so (C ABI, include/mocohip.h); this package is the
host-side mirror of the reference's MocoProblem / MocoSolver interface and
the model compiler that feeds the C ABI.
"""
from .model import (Axis, Body, Coordinate, CoordinateActuator, DataTable,  # noqa: F401
                    DeGrooteFregly2016Muscle, ExternalForce, Function, Joint,
                    Model, PathPoint)
from .problem import (MocoBounds, MocoControlGoal, MocoFinalTimeGoal,  # noqa: F401
                      MocoProblem, MocoStateTrackingGoal, MocoSumSquaredStateGoal)
from .solver import HipNLP, MocoHipSolver, MocoStudy  # noqa: F401
