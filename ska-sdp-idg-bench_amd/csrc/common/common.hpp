// common.hpp -- environment configuration, reporting and the work model.
//
// Entry points of the reference's app/common/common.{hpp,cpp}:10-159:
// get_env_var, report / report_csv (same stdout and CSV formats) and the
// flops_gridder / bytes_gridder work model that defines GFLOP/s, GB/s and the
// roofline numbers (the degridder reuses the gridder model, exactly as the
// reference does at app/HIP/util.cpp:337-343).
#pragma once

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "init.hpp"
#include "parameters.hpp"
#include "print.hpp"

unsigned roundToPowOf2(unsigned number);

unsigned long get_env_var(const char *env_var, unsigned long default_value);

std::string get_env_var(const char *env_var, std::string default_value);

void report(std::string name, double seconds = 0, double gflops = 0,
            double gbytes = 0, double mvis = 0, double joules = 0);

void report_csv(std::string name, std::string device_name = "",
                std::string file_extension = "", double seconds = 0,
                double gflops = 0, double gbytes = 0, double mvis = 0,
                double joules = 0);

uint64_t flops_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                       uint64_t nr_subgrids, uint64_t subgrid_size,
                       uint64_t nr_correlations);

uint64_t bytes_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                       uint64_t nr_subgrids, uint64_t subgrid_size,
                       uint64_t nr_correlations);
