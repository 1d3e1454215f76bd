/* ws_hip.h -- C ABI of the MI355X-native weather-sim time-step library (libws_hip.so).
 *
 * This is the drop-in boundary for the reference's weather-sim hot path
 * (/root/reference/src/weather-sim). Every entry point is `extern "C"`, takes plain
 * pointers / sizes, returns an int status (WS_OK == 0) and never throws; the message of
 * the last failure on the calling thread is available from ws_last_error(). No torch or
 * C++ types cross the boundary. All compute runs as hand-written HIP kernels on gfx950;
 * there is no CPU fallback: without a HIP device every creating call fails with
 * WS_ERR_DEVICE.
 *
 * Reference interfaces replaced (paths relative to src/weather-sim/cpp):
 *   ws_config_t                   SimulationConfig           include/weather_sim/weather_sim.hpp:155-191
 *   ws_metrics_t                  PerformanceMetrics         include/weather_sim/weather_sim.hpp:196-223
 *   ws_grid_*                     WeatherGrid                include/weather_sim/weather_sim.hpp:254-412,
 *                                                            src/weather_grid.cpp:15-142, and the pybind
 *                                                            field copies src/python_bindings.cpp:22-114,240-284
 *   ws_grid_apply_initial_condition  InitialCondition::initialize  src/initial_conditions.cpp:48-608
 *   ws_sim_*                      WeatherSimulation          include/weather_sim/weather_sim.hpp:417-544,
 *                                                            src/weather_simulation.cpp:17-158
 *   ws_adapter_*                  KernelAdapter (plugin API) include/weather_sim/gpu_adaptability.hpp:242-329
 *   ws_launch_shallow_water_kernel   launchShallowWaterKernel   src/kernels/shallow_water_kernels.cu:704-719
 *   ws_launch_diagnostics_kernels    launchDiagnosticsKernels   src/kernels/shallow_water_kernels.cu:830-840
 *   ws_device_info / ws_is_available AdaptiveKernelManager::getDeviceCapabilities / isCudaAvailable
 *                                                            include/weather_sim/gpu_adaptability.hpp:128-237
 *   ws_comm_* / ws_sim_create_slab   (new: the reference has no distributed path)
 *
 * Environment switches read by the library (all optional; everything else is an argument):
 *   WS_NUMERICS=exact|fast    numerics of the fused kernels at creation (ws_sim_set_numerics)
 *   WS_FUSED=0                per-stage kernels instead of the fused step kernel
 *   WS_KERNEL=dppy|x2y|pc|pc2|lds (pin the fused-kernel variant)     } each also settable per
 *   WS_TB=1|2|4|8             pin the steps per fused launch    } simulation with
 *   WS_SEG_ROWS=n             pin the rows per kernel segment   } ws_sim_pin_variant
 *   WS_AUTOTUNE=0|1|2         variant autotuner off / on (default) / on + print its table
 *   WS_TUNE_CACHE=path        append / reuse autotune choices across processes
 *   WS_SLAB_OVERLAP=0|1       fix the slab overlap schedule (default: chosen from a measured
 *                             halo exchange, ws_sim_set_slab_schedule)
 */
#ifndef WS_HIP_H
#define WS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WS_ABI_VERSION 2

/* status codes */
enum {
    WS_OK = 0,
    WS_ERR_INVALID = 1,     /* bad argument (reference: std::invalid_argument -> ValueError) */
    WS_ERR_DEVICE = 2,      /* HIP runtime / no device (reference: CUDA_CHECK -> false) */
    WS_ERR_SHAPE = 3,       /* array shape mismatch (reference setters: std::runtime_error) */
    WS_ERR_UNSUPPORTED = 4,
    WS_ERR_COMM = 5         /* RCCL failure */
};

/* field ids (WeatherGrid members, weather_sim.hpp:403-411) */
enum {
    WS_FIELD_U = 0, WS_FIELD_V = 1, WS_FIELD_H = 2, WS_FIELD_P = 3,
    WS_FIELD_T = 4, WS_FIELD_Q = 5, WS_FIELD_VORTICITY = 6, WS_FIELD_DIVERGENCE = 7
};

/* element types */
enum { WS_F32 = 0, WS_F64 = 1 };

/* enum values identical to weather_sim.hpp:30-76 */
enum { WS_MODEL_SHALLOW_WATER = 0, WS_MODEL_BAROTROPIC = 1, WS_MODEL_PRIMITIVE_EQUATIONS = 2, WS_MODEL_GENERAL = 3 };
enum { WS_EULER = 0, WS_RK2 = 1, WS_RK4 = 2, WS_ADAMS_BASHFORTH = 3, WS_SEMI_IMPLICIT = 4 };
enum { WS_BACKEND_CUDA = 0, WS_BACKEND_CPU = 1, WS_BACKEND_HYBRID = 2, WS_BACKEND_ADAPTIVE_HYBRID = 3 };

/* SimulationConfig (weather_sim.hpp:155-191). Scalars are passed as double and rounded to
 * the simulation precision (fp32 unless double_precision != 0) exactly as the reference
 * stores them in scalar_t. output_path stays on the host side of the boundary. */
typedef struct ws_config {
    int32_t model;
    int32_t grid_type;
    int32_t integration_method;
    int32_t boundary_condition;
    int32_t grid_width;
    int32_t grid_height;
    int32_t num_levels;          /* >1: L independent 2-D levels, fields are [L][H][W] */
    double dx, dy, dt;
    double gravity, coriolis_f, beta, viscosity, diffusivity;
    int32_t compute_backend;
    int32_t double_precision;    /* honoured: 0 -> fp32 (bitwise = reference), 1 -> fp64 */
    int32_t device_id;
    int32_t num_threads;
    double max_time;
    int32_t max_steps;
    int32_t output_interval;
    uint32_t random_seed;
} ws_config_t;

/* PerformanceMetrics (weather_sim.hpp:196-223). Times are device-event milliseconds
 * (not integer-truncated). */
typedef struct ws_metrics {
    double total_time_ms;
    double compute_time_ms;
    double memory_transfer_time_ms;
    double io_time_ms;
    int32_t num_steps;
} ws_metrics_t;

/* DeviceCapabilities (gpu_adaptability.hpp:35-88), filled for the HIP device */
typedef struct ws_device_info {
    char device_name[256];
    char arch[64];               /* e.g. "gfx950" */
    int32_t compute_capability_major, compute_capability_minor;
    int32_t multiprocessors;     /* CUs */
    int32_t cuda_cores;          /* stream processors = CUs * 64 */
    int64_t global_memory;       /* bytes */
    int32_t shared_memory_per_block;
    int32_t max_threads_per_block;
    int32_t max_threads_per_multiprocessor;
    int32_t clock_rate_khz;
    int32_t memory_clock_rate_khz;
    int32_t memory_bus_width;
    int32_t wavefront_size;
} ws_device_info_t;

typedef struct ws_grid ws_grid_t;
typedef struct ws_sim ws_sim_t;

const char* ws_last_error(void);
int ws_abi_version(void);
int ws_is_available(int32_t* available);
int ws_device_count(int32_t* count);
int ws_device_info(int32_t device, ws_device_info_t* out);
/* hipMemGetInfo of a device (the benchmark harness's device-memory figure) */
int ws_device_memory(int32_t device, int64_t* free_bytes, int64_t* total_bytes);
void ws_config_default(ws_config_t* cfg);

/* ---- WeatherGrid ---------------------------------------------------------------- */
int ws_grid_create(int32_t width, int32_t height, int32_t num_levels, int32_t dtype, int32_t device,
                   ws_grid_t** out);
int ws_grid_destroy(ws_grid_t* grid);
int ws_grid_reset(ws_grid_t* grid);
int ws_grid_get_dims(const ws_grid_t* grid, int32_t* width, int32_t* height, int32_t* num_levels,
                     int32_t* dtype);
int ws_grid_set_spacing(ws_grid_t* grid, double dx, double dy);
int ws_grid_get_spacing(const ws_grid_t* grid, double* dx, double* dy);
/* Copy a (height, width) C-contiguous host array of `dtype` into / out of one level of a
 * field (level = -1: all levels, host array (num_levels, height, width)). A dtype
 * different from the grid's is converted like a C cast. Reading VORTICITY/DIVERGENCE
 * first materialises pending diagnostics (see ws_grid_calculate_diagnostics). */
int ws_grid_set_field(ws_grid_t* grid, int32_t field, int32_t level, const void* host, int32_t height,
                      int32_t width, int32_t dtype);
int ws_grid_get_field(ws_grid_t* grid, int32_t field, int32_t level, void* host, int32_t height,
                      int32_t width, int32_t dtype);
/* Device address / row pitch (elements) / level stride (elements) of a field, for
 * zero-copy interop (e.g. torch.from_dlpack-free views). */
int ws_grid_device_field(ws_grid_t* grid, int32_t field, void** dptr, int64_t* pitch, int64_t* level_stride);
/* Vorticity / divergence (weather_grid.cpp:82-121). Marks them due; the kernel runs when
 * they are read (lazy), so a run() of N steps launches no diagnostics kernel. */
int ws_grid_calculate_diagnostics(ws_grid_t* grid);
/* InitialCondition::initialize(grid) for the registered names (initial_conditions.cpp:611-666):
 * "uniform"(u,v,h,p,t,q) "random"(seed,amplitude) "zonal_flow"(u_max,h_mean,beta)
 * "vortex"(x_center,y_center,radius,strength,h_mean) "jet_stream"(y_center,width,strength,h_mean)
 * "breaking_wave"(amplitude,wavelength,h_mean) "front"(y_position,width,temp_difference,wind_shear)
 * "mountain"(x_center,y_center,radius,height,u_base) "atmospheric_profile"(sparam = profile name).
 * Missing trailing params take the reference defaults. level = -1 applies to every level. */
int ws_grid_apply_initial_condition(ws_grid_t* grid, const char* name, const double* params, int32_t nparams,
                                    const char* sparam, int32_t level);

/* ---- WeatherSimulation ---------------------------------------------------------- */
int ws_sim_create(const ws_config_t* cfg, ws_sim_t** out);
int ws_sim_destroy(ws_sim_t* sim);
/* which = 0: current grid, 1: next grid. The handle is a stable slot: after a step the
 * simulation's current grid is the other slot (reference stale-handle semantics,
 * SURVEY Appendix C.7). Grids are owned by the simulation. */
int ws_sim_grid(ws_sim_t* sim, int32_t which, ws_grid_t** out);
/* initialize() minus the IC: time = step = 0, metrics reset, current grid reset()
 * (weather_simulation.cpp:46-66); the caller applies the IC to ws_sim_grid(sim, 0). */
int ws_sim_initialize(ws_sim_t* sim);
int ws_sim_step(ws_sim_t* sim);
/* run(n) (weather_simulation.cpp:68-103): stops after the step at which t >= max_time.
 * One call launches all steps on the device; *steps_taken may be NULL. */
int ws_sim_run(ws_sim_t* sim, int32_t num_steps, int32_t* steps_taken);
int ws_sim_run_until(ws_sim_t* sim, double max_time, int32_t* steps_taken);
int ws_sim_get_time(const ws_sim_t* sim, double* t);
int ws_sim_get_step(const ws_sim_t* sim, int32_t* step);
int ws_sim_get_dt(const ws_sim_t* sim, double* dt);
int ws_sim_set_dt(ws_sim_t* sim, double dt);
int ws_sim_get_config(const ws_sim_t* sim, ws_config_t* cfg);
int ws_sim_get_metrics(const ws_sim_t* sim, ws_metrics_t* m);
int ws_sim_reset_metrics(ws_sim_t* sim);
int ws_sim_synchronize(ws_sim_t* sim);
/* Device milliseconds of the last ws_sim_run / ws_sim_run_until (hipEvents on the sim's
 * stream) and the number of stage kernels it launched. */
int ws_sim_last_run_stats(const ws_sim_t* sim, double* device_ms, int64_t* kernel_launches);
/* Test hook: the next ws_sim_run / ws_sim_step fails with WS_ERR_DEVICE right after its
 * `after_launches`-th step launch (once; < 0 disarms) -- how the tests reach a run's error
 * path (state left consistent: the completed launches' steps, time and PE T / P drift). */
int ws_sim_inject_failure(ws_sim_t* sim, int32_t after_launches);

/* ---- KernelAdapter plugin API (gpu_adaptability.hpp:242-329) --------------------- */
/* One full forward-Euler step in -> out (the semantics of the reference's fused
 * shallowWaterStepKernel_*), gravity / coriolis_f explicit, dx/dy from `in`. Writes u,v,h
 * (+T,P for the PE model) of `out` and marks its diagnostics due. *ms = device time. */
int ws_adapter_execute_shallow_water_step(ws_grid_t* in, ws_grid_t* out, double dt, double gravity,
                                          double coriolis_f, double* ms);
int ws_adapter_execute_barotropic_step(ws_grid_t* in, ws_grid_t* out, double dt, double gravity,
                                       double coriolis_f, double* ms);
int ws_adapter_execute_primitive_equations_step(ws_grid_t* in, ws_grid_t* out, double dt, double gravity,
                                                double coriolis_f, double* ms);
int ws_adapter_execute_gcm_step(ws_grid_t* in, ws_grid_t* out, double dt, double gravity, double coriolis_f,
                                double* ms);
int ws_adapter_calculate_diagnostics(ws_grid_t* grid, double* ms);

/* ---- raw-pointer kernel ABI (shallow_water_kernels.cu:704-719, :830-840) ---------- */
/* Caller-owned device buffers, row pitch in elements (>= width), one level, stream may
 * be NULL (default stream). Asynchronous; returns WS_OK or WS_ERR_* on a launch error. */
int ws_launch_shallow_water_kernel(const void* d_u, const void* d_v, const void* d_h, void* d_u_out,
                                   void* d_v_out, void* d_h_out, int32_t width, int32_t height, int64_t pitch,
                                   double dt, double gravity, double dx, double dy, double coriolis_f,
                                   int32_t dtype, void* stream);
int ws_launch_diagnostics_kernels(const void* d_u, const void* d_v, void* d_vorticity, void* d_divergence,
                                  int32_t width, int32_t height, int64_t pitch, double dx, double dy,
                                  int32_t dtype, void* stream);

/* ---- slab decomposition over RCCL (new) ----------------------------------------- */
#define WS_COMM_ID_BYTES 128
int ws_comm_get_unique_id(uint8_t id[WS_COMM_ID_BYTES]);
/* One rank of a y-slab decomposition of the global grid described by cfg. Rank r owns
 * rows [row0, row0 + rows) (balanced split, returned); halo rows are exchanged with
 * ncclSend/ncclRecv between neighbouring ranks (id: from ws_comm_get_unique_id on one rank,
 * the same bytes on every rank; NULL is an error). Fields set / read through the slab's
 * grids are the local rows only. Results are bitwise identical to one GPU. */
int ws_sim_create_slab(const ws_config_t* cfg, int32_t rank, int32_t nranks, const uint8_t id[WS_COMM_ID_BYTES],
                       ws_sim_t** out, int32_t* row0, int32_t* rows);
/* Measurement aid: rank `rank`'s slab WITHOUT a communicator. Its halo exchanges are
 * replaced by a device-side wait of xfer_us microseconds (the direct transport) or the
 * pack / unpack kernels around that wait (the packed one), so one process can time one
 * rank's whole schedule of an N-rank decomposition on one GPU; the halo rows keep what they
 * hold, so results differ from the decomposed run (timing only). nranks >= 2. */
int ws_sim_create_slab_emulated(const ws_config_t* cfg, int32_t rank, int32_t nranks, double xfer_us,
                                ws_sim_t** out, int32_t* row0, int32_t* rows);

/* Slab group: the same y-slab decomposition and step schedule (interior segments while the
 * halo moves, then edge segments) inside ONE process on one device, halo rows moved by
 * device copies. Used to verify the decomposition bitwise against the single-domain run
 * on a single GPU. Slabs are owned by the group and step only through ws_group_run. */
typedef struct ws_group ws_group_t;
int ws_group_create(const ws_config_t* cfg, int32_t nslabs, ws_group_t** out);
int ws_group_destroy(ws_group_t* group);
int ws_group_slab(ws_group_t* group, int32_t rank, ws_sim_t** sim, int32_t* row0, int32_t* rows);
int ws_group_run(ws_group_t* group, int32_t num_steps, int32_t* steps_taken);

/* Multi-GPU simulation in ONE process (new; the reference's WeatherSimulation
 * takes one device, weather_sim.hpp:180): the y-slab decomposition of cfg's global grid over
 * `ndevices` devices, slab r on devices[r]. Distinct devices: each slab is a full rank of the
 * RCCL decomposition (exactly ws_sim_create_slab's, communicators created together), driven
 * by a host thread of its own with its device current; ws_multi_run / _step / _run_until /
 * _cfl run every rank at once. All devices equal (ndevices > 1): the slabs share that device
 * and a slab group (device-copy halos) runs them. Slab handles (ws_multi_slab) are owned by
 * the multi simulation: read / write their grids and query them, step only through ws_multi_*.
 * Results are bitwise identical to one domain. */
typedef struct ws_multi ws_multi_t;
int ws_multi_create(const ws_config_t* cfg, const int32_t* devices, int32_t ndevices, ws_multi_t** out);
int ws_multi_destroy(ws_multi_t* multi);
/* *shared_device = 1 when the slabs share one device (slab group transport) */
int ws_multi_size(const ws_multi_t* multi, int32_t* nslabs, int32_t* shared_device);
int ws_multi_slab(ws_multi_t* multi, int32_t rank, ws_sim_t** sim, int32_t* row0, int32_t* rows);
int ws_multi_step(ws_multi_t* multi);
int ws_multi_run(ws_multi_t* multi, int32_t num_steps, int32_t* steps_taken);
int ws_multi_run_until(ws_multi_t* multi, double max_time, int32_t* steps_taken);
/* CFL of the global state (max over slabs; see ws_sim_cfl) */
int ws_multi_cfl(ws_multi_t* multi, double* cfl, double* per_level, int32_t nlevels, double* ms);
int ws_multi_synchronize(ws_multi_t* multi);
/* After writing fields outside run() (an initial condition, field setters): refresh every
 * slab's one-row u, v halo from its neighbours (collective) so vorticity / divergence read
 * next are correct at the slab seams; run() does this itself at its end. */
int ws_multi_exchange_diag_halo(ws_multi_t* multi);

/* The halo exchange plan of rank `rank` (new; the reference has no distributed path): the
 * byte ranges a slab's exchange of `depth` rows of `nfields` level-stacked fields moves.
 * Offsets are relative to a field's row 0 of level 0 in the slab-grid layout (`pitch`
 * elements per row, `level_stride` elements per level, 24 halo rows above and below each
 * level). Per neighbour there is ONE message: its send segments (kind 0) concatenated in
 * plan order (field-major, then level; msg_offset = position in the message), received
 * into the receive segments (kind 1) in the same order. ws_sim_create_slab's RCCL exchange
 * and ws_group_run's device copies both execute exactly this plan: with at most 4 segments
 * per neighbour (SWE: u, v, h) every segment moves by its own send / receive straight
 * between the field rows (the direct transport); with more (PE: 3 x levels) they are packed
 * into the one message, moved and unpacked.
 * out = NULL: only count / pitch / level_stride. */
typedef struct {
    int32_t peer;        /* neighbour rank */
    int32_t kind;        /* 0 = send, 1 = receive */
    int32_t field;       /* index into the exchanged fields (u, v, h: 0, 1, 2) */
    int32_t level;
    int64_t offset;      /* bytes from the field's row 0 of level 0 */
    int64_t bytes;
    int64_t msg_offset;  /* bytes into the message exchanged with `peer` */
} ws_xfer_t;
int ws_slab_exchange_plan(int32_t width, int32_t rows, int32_t levels, int32_t dtype, int32_t rank, int32_t nranks,
                          int32_t nfields, int32_t depth, ws_xfer_t* out, int32_t capacity, int32_t* count,
                          int64_t* pitch, int64_t* level_stride);

/* Row range [row0, row0 + rows) of rank `rank` in the balanced split of `height` rows. */
int ws_slab_partition(int32_t height, int32_t rank, int32_t nranks, int32_t* row0, int32_t* rows);
/* Collectives on the slab communicator (max over ranks of one double; barrier). On a
 * single-GPU simulation they are local no-ops. */
int ws_sim_comm_allreduce_max(ws_sim_t* sim, double value, double* out);
int ws_sim_comm_barrier(ws_sim_t* sim);

/* ---- physics-mode barotropic vorticity model (new) ------------------ */
/* BASELINE config C3 names a "Jacobian + Laplacian" barotropic model; the reference has
 * none (its Barotropic model runs the SWE tendencies, weather_simulation.cpp:542-560, which
 * ws_sim_* reproduces bit for bit). This is that model, defined by oracle/bvort_oracle.py:
 * doubly periodic, d(zeta)/dt = -J(psi, zeta) - beta psi_x + nu lap(zeta), lap(psi) = zeta
 * (Arakawa Jacobian, spectral Poisson via hipFFT). From cfg it reads grid_width/height, dx,
 * dy, dt, beta, viscosity (the SimulationConfig fields the reference never reads,
 * weather_sim.hpp:176-178), integration_method (Euler / RK2 / classical RK4; others run
 * Euler), double_precision and device_id. */
typedef struct ws_bvort ws_bvort_t;
int ws_bvort_create(const ws_config_t* cfg, ws_bvort_t** out);
/* poisson: WS_POISSON_AUTO = the LDS-resident FFT passes on power-of-two grids up to 4096,
 * hipFFT's 2-D plans otherwise; WS_POISSON_HIPFFT = hipFFT always (cross-check). */
#define WS_POISSON_AUTO 0
#define WS_POISSON_HIPFFT 1
int ws_bvort_create_poisson(const ws_config_t* cfg, int32_t poisson, ws_bvort_t** out);
int ws_bvort_destroy(ws_bvort_t* model);
/* (height, width) C-contiguous host array, fp32 or fp64 (converted like a C cast) */
int ws_bvort_set_vorticity(ws_bvort_t* model, const void* host, int32_t height, int32_t width, int32_t dtype);
/* which: 0 vorticity, 1 streamfunction, 2 u = -psi_y, 3 v = psi_x; dtype = the model's */
int ws_bvort_get_field(ws_bvort_t* model, int32_t which, void* host, int32_t height, int32_t width, int32_t dtype);
/* n steps on the device, one host synchronisation at the end */
int ws_bvort_run(ws_bvort_t* model, int32_t num_steps);
int ws_bvort_get_state(const ws_bvort_t* model, double* time, int32_t* step, double* last_run_ms,
                       int64_t* last_run_launches);
/* y-slab decomposition of the vorticity model around its periodic ring (new; LDS-FFT Poisson
 * path only: power-of-two width and height, a power-of-two slab count n with height % (2 n) ==
 * 0 and (width / 2) % n == 0). The row FFTs stay local to a slab; the spectrum is transposed
 * in blocks of width / (2 n) columns to the column pass and back (slab q solves global columns
 * [q nc, (q + 1) nc)), and the stencil reads one halo row of psi and zeta from the ring
 * neighbours. Every pass is the single domain's on the same rows / columns: results are
 * bitwise identical to ws_bvort_create's. ws_bvort_create_multi: ONE model over `ndevices`
 * slabs in this process, slab r on devices[r] (repeats share a device; transposes and halos by
 * the process's own copies); used like ws_bvort_create's (whole fields in and out). */
int ws_bvort_create_multi(const ws_config_t* cfg, int32_t poisson, const int32_t* devices, int32_t ndevices,
                          ws_bvort_t** out);
/* One rank of a process-per-GPU decomposition (device cfg->device_id): transposes by RCCL
 * send / receive per block, halos by the periodic plan of ws_lpe_exchange_plan's kind; set /
 * get take the rank's rows (height = rows); run() and field reads that need psi are
 * collective. */
int ws_bvort_create_slab(const ws_config_t* cfg, int32_t poisson, int32_t rank, int32_t nranks,
                         const uint8_t id[WS_COMM_ID_BYTES], ws_bvort_t** out, int32_t* row0, int32_t* rows);
int ws_bvort_layout(const ws_bvort_t* model, int32_t* nslabs, int32_t* row0, int32_t* rows);

/* ---- physics-mode layered primitive-equation model (new) ----------- */
/* BASELINE config C4 names a 3-D primitive-equation stencil with vertical columns; the
 * reference has none (its PE model runs the SWE tendencies level by level, which ws_sim_*
 * reproduces bit for bit). This is that model, defined by oracle/layered_pe_oracle.py:
 * hydrostatic primitive equations in isopycnal coordinates -- num_levels stacked layers of
 * constant density (k = 0 on top), flat bottom, doubly periodic -- coupled through the
 * Montgomery potential M_0 = g eta_0, M_k = M_{k-1} + reduced_gravity * eta_k (eta_k = height
 * of layer k's top). From cfg it reads grid_width/height, num_levels, dx, dy, dt, gravity,
 * coriolis_f, integration_method (Euler / RK2 / classical RK4), double_precision and
 * device_id; any number of levels. Fields are (num_levels, height, width) arrays: 0 u, 1 v,
 * 2 h (thickness). */
typedef struct ws_lpe ws_lpe_t;
int ws_lpe_create(const ws_config_t* cfg, double reduced_gravity, ws_lpe_t** out);
int ws_lpe_destroy(ws_lpe_t* model);
int ws_lpe_set_field(ws_lpe_t* model, int32_t field, const void* host, int32_t levels, int32_t height,
                     int32_t width, int32_t dtype);
int ws_lpe_get_field(ws_lpe_t* model, int32_t field, void* host, int32_t levels, int32_t height, int32_t width,
                     int32_t dtype);
int ws_lpe_run(ws_lpe_t* model, int32_t num_steps);
int ws_lpe_get_state(const ws_lpe_t* model, double* time, int32_t* step, double* last_run_ms,
                     int64_t* last_run_launches);
/* y-slab decomposition of the layered model around its periodic ring (new): slab r owns the
 * rows [row0, row0 + rows) of the balanced split (ws_slab_partition) with one halo row above
 * and below every level, refreshed from the ring neighbours (slab 0's upper neighbour is the
 * last slab) before every RK stage. Results are bitwise identical to ws_lpe_create's.
 * ws_lpe_create_multi: ONE model over `ndevices` slabs in this process, slab r on devices[r]
 * (entries may repeat: slabs sharing a device); halos pulled from the neighbours' memory by a
 * copy kernel (peer access between distinct devices, else the runtime's 2-D copies). The
 * handle is used like ws_lpe_create's: set / get_field take the whole (levels, height, width)
 * field, run steps every slab. */
int ws_lpe_create_multi(const ws_config_t* cfg, double reduced_gravity, const int32_t* devices, int32_t ndevices,
                        ws_lpe_t** out);
/* One rank of a process-per-GPU decomposition (device cfg->device_id): halos over RCCL
 * (id from ws_comm_get_unique_id, the same bytes on every rank) with the periodic plan of
 * ws_lpe_exchange_plan. Its set / get_field take the rank's own rows, (levels, rows, width);
 * run() is collective. */
int ws_lpe_create_slab(const ws_config_t* cfg, double reduced_gravity, int32_t rank, int32_t nranks,
                       const uint8_t id[WS_COMM_ID_BYTES], ws_lpe_t** out, int32_t* row0, int32_t* rows);
/* slabs of the decomposition (1: one domain) and this handle's global row range */
int ws_lpe_layout(const ws_lpe_t* model, int32_t* nslabs, int32_t* row0, int32_t* rows);
/* The periodic halo plan of rank `rank` (fields u, v, h; depth 1): like ws_slab_exchange_plan,
 * but the ring closes (every rank has both neighbours when nranks > 1; with two ranks they are
 * the same peer) and the slab layout is unpadded (pitch = width, level stride returned =
 * (rows + 2) x width, one halo row). The transport posts the sends to side 0 (upper) and
 * side 1 (lower), then the receives from side 1 and side 0, so a pair's k-th send meets the
 * peer's k-th receive. */
int ws_lpe_exchange_plan(int32_t width, int32_t rows, int32_t levels, int32_t dtype, int32_t rank, int32_t nranks,
                         ws_xfer_t* out, int32_t capacity, int32_t* count, int64_t* level_stride);

/* ---- per-kernel timing (measurement) --------------------------------------------- */
/* When enabled, ws_sim_run / ws_sim_step time their kernels with hipEvents on the
 * simulation's stream: a run whose steps are one fused launch each (and nothing else on
 * the stream) is timed as a whole and attributed per launch (no events between the
 * launches); otherwise every 8th fused launch (or every per-stage kernel of the fallback
 * path) is bracketed by events. kind = stage index within the step (0..3 for RK4; 0 for
 * the fused kernel). The statistics reset when timing is (re-)enabled. bytes_per_launch
 * is the algorithmic HBM traffic of one launch (SURVEY §8(d) words x cells x element size;
 * the fused kernel: 6 words).
 * enable = 0: off; 1: on; n > 1: on, with events for n launches created up front. */
int ws_sim_set_kernel_timing(ws_sim_t* sim, int32_t enable);
int ws_sim_kernel_timing(const ws_sim_t* sim, int32_t kind, int64_t* launches, double* total_ms,
                         double* bytes_per_launch);

/* The fused step-kernel variant in use: kernel 0 = LDS workgroups (256 columns), 4 = DPP
 * waves (64 columns per wave) with y rows staged by LDS-DMA and read from LDS in place,
 * 5 = the same with an adjacent column pair per lane (128 columns per wave), 6 = the DPP
 * kernel's two-step launch split over a producer wave (the first step) and a consumer wave
 * (the second) per strip, handing rows over through LDS (its one-step launches are kernel
 * 4's), 7 = the same split of kernel 5 (column pairs), -1 = per-stage kernels (ids 1-3 are retired variants); seg_rows = output rows per segment (or -r - 1: r chains per SIMD), out_cols =
 * output columns per strip (a multiple of the 128-byte line when the strips are
 * line-aligned). Chosen by timing every variant on the real grid at the first run (all give
 * identical results), unless WS_KERNEL / WS_SEG_ROWS / ws_sim_pin_variant fix it. The
 * choice is cached per process by (grid shape, levels, precision, model, integrator,
 * numerics, slab position and block), and a slab decomposition uses rank 0's choice on every
 * rank. */
int ws_sim_fused_variant(const ws_sim_t* sim, int32_t* kernel, int32_t* seg_rows, int32_t* out_cols);

/* Pin (part of) the fused-kernel variant of one simulation; -1 leaves a part to the
 * autotuner, which then times only candidates that agree with the pinned parts (a pinned
 * kernel gets its own best steps per launch, segment length and alignment). kernel:
 * WS_KERNEL_LDS / _DPPY / _X2Y / _PC / _PC2; steps_per_launch: 1, 2, 4 or 8 (the split variants _PC /
 * _PC2 advance two steps per launch: 1 is rejected, -1 means 2; _LDS one: 2 and 4 are rejected;
 * 4 = four steps where the kernel takes them -- Euler / RK2 with _DPPY, or _X2Y in fp32 -- else
 * two, as WS_TB=4; 8 = eight for Euler on the same kernels, else the largest they take);
 * seg_rows: output rows per segment, or -2 .. -9 = the chain schedule with 1 .. 8 cost-balanced
 * chains (one wave each) per SIMD; align: 1 = strip output windows on whole 128-byte lines.
 * The WS_KERNEL / WS_TB / WS_SEG_ROWS environment pins are process-wide and switch tuning off
 * (what they leave free takes its default; WS_KERNEL=pc|pc2 implies WS_TB=2). */
#define WS_KERNEL_LDS 0
#define WS_KERNEL_DPPY 4
#define WS_KERNEL_X2Y 5
#define WS_KERNEL_PC 6
#define WS_KERNEL_PC2 7
int ws_sim_pin_variant(ws_sim_t* sim, int32_t kernel, int32_t steps_per_launch, int32_t seg_rows, int32_t align);

/* Time steps per fused launch the simulation's run() uses where it can (new; temporal
 * blocking): 1, 2 = the dppy-family kernel advances two steps per launch (y_n read once,
 * y_{n+2} written once), 4 (Euler / RK2: four steps, y_n in and y_{n+4} out) or 8 (Euler).
 * Chosen by the autotuner (WS_TB=1|2|4|8 fixes it). A k-step launch runs only inside run() with >= k steps
 * left, inside a slab block with room for them (else 2, then 1), and with the configured
 * spacing on both grids; results are identical to one-step launches. */
int ws_sim_steps_per_launch(const ws_sim_t* sim, int32_t* steps);

/* Slab schedule (new: the reference has no distributed path): block = time steps per halo
 * exchange (deep halo of block x NST rows; 1 for a whole domain), overlap = 1 when run()
 * uses the overlap schedule -- each block's edge bands (the rows the neighbours need) on a
 * second HIP stream followed there by the halo exchange, the interior rows meanwhile on the
 * compute stream (bit-identical to the stream-ordered schedule).
 * Default (WS_OVERLAP_AUTO): at the first run rank 0 times the block's halo exchange on the
 * real communicator and every rank runs the overlap schedule iff that exchange takes longer
 * than the edge bands' measured cost (needs >= 3 x block x NST rows per slab); a slab group
 * (one process) overlaps whenever there is an interior. WS_SLAB_OVERLAP=0|1 fixes it.
 * ws_sim_set_slab_schedule: block (> 0; <= 0 keeps it; every rank must pass the same values)
 * and overlap mode; ws_sim_slab_exchange_us: the measured exchange (auto mode; -1 if none);
 * ws_sim_slab_trial_ms: the auto schedule's trial, ms per block period of each schedule
 * (ms[0] stream-ordered, ms[1] overlapped; max over ranks; -1 until a trial ran). The trial
 * keeps the overlap iff ms[1] < ms[0] * (1 - WS_OVERLAP_MARGIN): on a near-tie the
 * stream-ordered schedule (no cross-stream waits) stays. */
#define WS_OVERLAP_MARGIN 0.02
#define WS_OVERLAP_OFF 0
#define WS_OVERLAP_ON 1
#define WS_OVERLAP_AUTO 2
int ws_sim_slab_schedule(const ws_sim_t* sim, int32_t* block, int32_t* overlap);
int ws_sim_set_slab_schedule(ws_sim_t* sim, int32_t block, int32_t overlap);
int ws_sim_slab_exchange_us(const ws_sim_t* sim, double* us);
int ws_sim_slab_trial_ms(const ws_sim_t* sim, double* ms);

/* CFL number of the current state (new: the reference's dt is fixed and it has no CFL):
 * max over cells of max((|u| + sqrt(g h)) dt / dx, (|v| + sqrt(g h)) dt / dy), computed in
 * the simulation's precision by a device max-reduction (one pass over u, v, h; DPP wave
 * reductions); NaN if any cell is NaN or h < 0. *cfl = the maximum over all levels (and, on a
 * slab of a multi-GPU decomposition, over all ranks: an RCCL max-allreduce, so every rank
 * must call it); per_level (optional, nlevels >= num_levels entries) = per level; ms
 * (optional) = device time of the reduction kernels. */
int ws_sim_cfl(ws_sim_t* sim, double* cfl, double* per_level, int32_t nlevels, double* ms);
/* Waves per SIMD one launch of the fused step kernel in use holds (hipOccupancy of the
 * variant and steps per launch the autotuner chose; 0 for the per-stage kernels). */
int ws_sim_kernel_occupancy(const ws_sim_t* sim, int32_t* waves_per_simd);

/* ---- numerics mode of the fused step kernels ------------------------------------------
 * WS_NUMERICS_EXACT: the reference's arithmetic in the reference's evaluation order, no
 *   contraction: bit-for-bit equal to the CPU solver (weather_simulation.cpp:160-540).
 * WS_NUMERICS_FAST: the same tendencies and integrators re-associated for the hardware
 *   (fused multiply-adds, the 1/(2dx) factor folded into the update constants, RK4's final
 *   combination as y + dt/3 ((k2 + k3) + k4)); isotropic spacing only (dx == dy: otherwise
 *   the kernels stay exact). Results differ from the reference by rounding only
 *   (north_star tolerance for fp64: <= 1e-10 relative L2; measured in
 *   tests/test_gpu_numerics.py).
 * Default: FAST for fp64 simulations, EXACT for fp32; the environment variable
 * WS_NUMERICS=exact|fast overrides the default at creation. The per-stage fallback kernels
 * (WS_FUSED=0) and the adapter / raw-launcher entry points are always exact. */
#define WS_NUMERICS_EXACT 0
#define WS_NUMERICS_FAST 1
int ws_sim_set_numerics(ws_sim_t* sim, int32_t mode);
int ws_sim_get_numerics(const ws_sim_t* sim, int32_t* mode);

#ifdef __cplusplus
}
#endif
#endif /* WS_HIP_H */
