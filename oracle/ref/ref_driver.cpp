// Test-infrastructure driver for the REFERENCE weather-sim CPU solver.
//
// This file is NOT part of the product. It is compiled by oracle/ref/build_ref.py
// together with the reference's own weather_grid.cpp / weather_simulation.cpp /
// initial_conditions.cpp (taken from /root/reference, mechanically compile-fixed in a
// scratch directory, never copied into this repo) to produce oracle/_ref/ws_ref_{f32,f64}.
// Those binaries generate the golden fixtures in tests/golden/ and may serve as the
// "reference" CPU baseline in bench.py.
//
// It drives the public C++ API exactly as pyweather_sim does
// (reference: src/weather-sim/cpp/src/python_bindings.cpp:338-353):
//   WeatherSimulation(config) -> setInitialCondition -> initialize -> step/run/runUntil,
// then dumps the current grid's fields (getVelocityField/getHeightField/...).
//
// Spec file: one command per line.
//   cfg <key> <value>           SimulationConfig field (before "create")
//   create                      construct WeatherSimulation
//   ic <name> <p0> <p1> ...     set an initial condition (constructor args, in order)
//   initialize
//   setfield <u|v|h|p|t|q> <path>   load W*H scalar_t from raw file into current grid
//   step <n> | run <n> | run_until <T> | set_dt <dt>
//   hold                        remember &getCurrentGrid() (stale-handle quirk)
//   snap <path> | snap_held <path>
//   time_run <n>                run(n) and print wall seconds (CPU baseline timing)
//   icband <name> <gW> <gH> <y0:rows,...> <prefix> [p0 p1 ...]
//                               evaluate IC <name> once on a standalone gW x gH WeatherGrid
//                               (global coordinates) and write, per band, rows
//                               [y0, y0 + rows) of u, v, h, p, t, q to
//                               <prefix>_<y0>_<field>.bin (the input of a band run:
//                               setfield them into a gW x rows simulation)
#include "weather_sim/weather_sim.hpp"
#include "weather_sim/initial_conditions.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

using namespace weather_sim;

static void dump(const WeatherGrid& g, const WeatherSimulation& sim, const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    int32_t hdr[4] = {0x57534731, g.getWidth(), g.getHeight(), (int32_t)sizeof(scalar_t)};
    std::fwrite(hdr, sizeof(hdr), 1, f);
    int32_t step = sim.getCurrentStep();
    double t = (double)sim.getCurrentTime();
    std::fwrite(&step, sizeof(step), 1, f);
    std::fwrite(&t, sizeof(t), 1, f);
    const size_t n = (size_t)g.getWidth() * g.getHeight();
    auto w = [&](const std::vector<scalar_t>& v) { std::fwrite(v.data(), sizeof(scalar_t), n, f); };
    w(g.getVelocityField().u);
    w(g.getVelocityField().v);
    w(g.getHeightField().data);
    w(g.getPressureField().data);
    w(g.getTemperatureField().data);
    w(g.getHumidityField().data);
    w(g.getVorticityField().data);
    std::fclose(f);
}

static void load(std::vector<scalar_t>& dst, const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    size_t got = std::fread(dst.data(), sizeof(scalar_t), dst.size(), f);
    std::fclose(f);
    if (got != dst.size()) { std::fprintf(stderr, "short read %s\n", path.c_str()); std::exit(2); }
}

static std::shared_ptr<InitialCondition> make_ic(const std::string& name, const std::vector<std::string>& a) {
    auto F = [&](size_t i, float d) { return i < a.size() ? (scalar_t)std::stod(a[i]) : (scalar_t)d; };
    if (name == "uniform") return std::make_shared<UniformInitialCondition>(F(0, 0), F(1, 0), F(2, 10), F(3, 1000), F(4, 300), F(5, 0));
    if (name == "random") return std::make_shared<RandomInitialCondition>(a.size() > 0 ? (unsigned)std::stoul(a[0]) : 0u, F(1, 1));
    if (name == "zonal_flow") return std::make_shared<ZonalFlowInitialCondition>(F(0, 10), F(1, 10), F(2, 0.1f));
    if (name == "vortex") return std::make_shared<VortexInitialCondition>(F(0, 0.5f), F(1, 0.5f), F(2, 0.1f), F(3, 10), F(4, 10));
    if (name == "jet_stream") return std::make_shared<JetStreamInitialCondition>(F(0, 0.5f), F(1, 0.1f), F(2, 10), F(3, 10));
    if (name == "breaking_wave") return std::make_shared<BreakingWaveInitialCondition>(F(0, 1), F(1, 0.2f), F(2, 10));
    if (name == "front") return std::make_shared<FrontInitialCondition>(F(0, 0.5f), F(1, 0.05f), F(2, 10), F(3, 5));
    if (name == "mountain") return std::make_shared<MountainInitialCondition>(F(0, 0.3f), F(1, 0.5f), F(2, 0.1f), F(3, 1), F(4, 5));
    if (name == "atmospheric_profile") return std::make_shared<AtmosphericProfileInitialCondition>(a.size() ? a[0] : std::string("standard"));
    std::fprintf(stderr, "unknown ic %s\n", name.c_str());
    std::exit(2);
}

int main(int argc, char** argv) {
    if (argc != 2) { std::fprintf(stderr, "usage: %s spec.txt\n", argv[0]); return 2; }
    std::ifstream in(argv[1]);
    SimulationConfig cfg;
    cfg.compute_backend = ComputeBackend::CPU;  // the only working backend
    cfg.random_seed = 0;
    std::unique_ptr<WeatherSimulation> sim;
    WeatherGrid* held = nullptr;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string cmd;
        if (!(ss >> cmd) || cmd[0] == '#') continue;
        if (cmd == "cfg") {
            std::string k, v;
            ss >> k >> v;
            if (k == "width") cfg.grid_width = std::stoi(v);
            else if (k == "height") cfg.grid_height = std::stoi(v);
            else if (k == "model") cfg.model = (SimulationModel)std::stoi(v);
            else if (k == "method") cfg.integration_method = (IntegrationMethod)std::stoi(v);
            else if (k == "dt") cfg.dt = (scalar_t)std::stod(v);
            else if (k == "dx") cfg.dx = (scalar_t)std::stod(v);
            else if (k == "dy") cfg.dy = (scalar_t)std::stod(v);
            else if (k == "gravity") cfg.gravity = (scalar_t)std::stod(v);
            else if (k == "coriolis_f") cfg.coriolis_f = (scalar_t)std::stod(v);
            else if (k == "max_time") cfg.max_time = (scalar_t)std::stod(v);
            else { std::fprintf(stderr, "unknown cfg %s\n", k.c_str()); return 2; }
        } else if (cmd == "create") {
            sim.reset(new WeatherSimulation(cfg));
        } else if (cmd == "ic") {
            std::string name, tok;
            std::vector<std::string> a;
            ss >> name;
            while (ss >> tok) a.push_back(tok);
            sim->setInitialCondition(make_ic(name, a));
        } else if (cmd == "initialize") {
            sim->initialize();
        } else if (cmd == "setfield") {
            std::string which, path;
            ss >> which >> path;
            WeatherGrid& g = sim->getCurrentGrid();
            if (which == "u") load(g.getVelocityField().u, path);
            else if (which == "v") load(g.getVelocityField().v, path);
            else if (which == "h") load(g.getHeightField().data, path);
            else if (which == "p") load(g.getPressureField().data, path);
            else if (which == "t") load(g.getTemperatureField().data, path);
            else if (which == "q") load(g.getHumidityField().data, path);
            else return 2;
        } else if (cmd == "step") {
            int n; ss >> n;
            for (int i = 0; i < n; ++i) sim->step();
        } else if (cmd == "run") {
            int n; ss >> n;
            sim->run(n);
        } else if (cmd == "run_until") {
            double t; ss >> t;
            sim->runUntil((scalar_t)t);
        } else if (cmd == "set_dt") {
            double t; ss >> t;
            sim->setDt((scalar_t)t);
        } else if (cmd == "hold") {
            held = &sim->getCurrentGrid();
        } else if (cmd == "snap") {
            std::string p; ss >> p;
            dump(sim->getCurrentGrid(), *sim, p);
        } else if (cmd == "snap_held") {
            std::string p; ss >> p;
            dump(*held, *sim, p);
        } else if (cmd == "icband") {
            std::string name, bands, prefix, tok;
            int gW, gH;
            ss >> name >> gW >> gH >> bands >> prefix;
            std::vector<std::string> a;
            while (ss >> tok) a.push_back(tok);
            WeatherGrid g(gW, gH);
            make_ic(name, a)->initialize(g);
            std::istringstream bs(bands);
            std::string b;
            while (std::getline(bs, b, ',')) {
                const int y0 = std::stoi(b.substr(0, b.find(':'))), rows = std::stoi(b.substr(b.find(':') + 1));
                if (y0 < 0 || rows <= 0 || y0 + rows > gH) { std::fprintf(stderr, "bad band %s\n", b.c_str()); return 2; }
                auto band = [&](const std::vector<scalar_t>& v, const char* f) {
                    const std::string path = prefix + "_" + std::to_string(y0) + "_" + f + ".bin";
                    FILE* o = std::fopen(path.c_str(), "wb");
                    if (!o) { std::perror(path.c_str()); std::exit(2); }
                    std::fwrite(v.data() + (size_t)y0 * gW, sizeof(scalar_t), (size_t)rows * gW, o);
                    std::fclose(o);
                };
                band(g.getVelocityField().u, "u");
                band(g.getVelocityField().v, "v");
                band(g.getHeightField().data, "h");
                band(g.getPressureField().data, "p");
                band(g.getTemperatureField().data, "t");
                band(g.getHumidityField().data, "q");
            }
        } else if (cmd == "time_run") {
            int n; ss >> n;
            auto t0 = std::chrono::steady_clock::now();
            sim->run(n);
            auto t1 = std::chrono::steady_clock::now();
            std::printf("TIME_RUN %d %.9f\n", sim->getCurrentStep(), std::chrono::duration<double>(t1 - t0).count());
        } else {
            std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
            return 2;
        }
    }
    return 0;
}
