"""weather_sim -- MI355X-native drop-in for the reference's weather-sim Python package.

Same public names as /root/reference/src/weather-sim/python/__init__.py (minus the
matplotlib visualization helpers, out of scope) and the pyweather_sim classes that
weather_simulation.py re-exports. Compute runs in hand-written HIP kernels on gfx950
through libws_hip.so; see DESIGN.md.
"""
from .weather_simulation import (  # noqa: F401
    AdaptiveKernelManager, AtmosphericProfileInitialCondition, BoundaryCondition, BreakingWaveInitialCondition,
    ComputeBackend, DeviceCapabilities, DeviceType, FrontInitialCondition, GridType, HIPKernelAdapter,
    InitialCondition, InitialConditionFactory, IntegrationMethod, JetStreamInitialCondition, KernelAdapter,
    KernelAdapterFactory, MountainInitialCondition, OutputConfig, OutputFormat, OutputManager, PerformanceMetrics,
    SlabGroup,
    MultiGPUSimulation,
    SlabbedGrid,
    SlabSimulation,
    new_comm_id,
    RandomInitialCondition, SimulationConfig, SimulationModel, UniformInitialCondition, VortexInitialCondition,
    WeatherGrid, WeatherSimulation, WeatherSimulationWrapper, ZonalFlowInitialCondition, create_initial_condition,
    get_available_initial_conditions, get_device_info, is_cuda_available, register_all_initial_conditions)
from .physics import BarotropicVorticityModel, LayeredPrimitiveEquationsModel  # noqa: F401
from .output import (  # noqa: F401
    CSVOutputManager, Snapshot, proto_classes, read_csv, weather_sim_result, weather_sim_update, write_csv)

__version__ = '0.1.0'
