// dft_processor_hip.cpp -- srsran::dft_processor over srs_amd_dft_run (see the header).
#include "dft_processor_hip.h"

#include "srsran_amd/ofdm.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

using namespace srsran;

namespace {

class dft_processor_hip : public dft_processor
{
public:
  dft_processor_hip(srs_amd_dft* d, const configuration& c) : dft(d), cfg(c), input(c.size), output(c.size) {}
  ~dft_processor_hip() override { srs_amd_dft_destroy(dft); }

  direction get_direction() const override { return cfg.dir; }
  unsigned  get_size() const override { return cfg.size; }
  span<cf_t> get_input() override { return input; }

  // dft_processor.h:66: the transform of get_input(), unnormalised (exp(-2 pi i n k / N) for DIRECT).
  span<const cf_t> run() override
  {
    if (srs_amd_dft_run(dft, reinterpret_cast<float*>(output.data()), reinterpret_cast<const float*>(input.data())) !=
        SRS_AMD_OK) {
      // the interface has no error path: report and hand back zeros rather than stale data
      std::fprintf(stderr, "dft_processor_hip: %s\n", srs_amd_last_error());
      std::fill(output.begin(), output.end(), cf_t());
    }
    return output;
  }

private:
  srs_amd_dft*      dft;
  configuration     cfg;
  std::vector<cf_t> input, output;
};

class dft_processor_factory_hip : public dft_processor_factory
{
public:
  explicit dft_processor_factory_hip(int device_) : device(device_) {}

  std::unique_ptr<dft_processor> create(const dft_processor::configuration& config) override
  {
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
      return nullptr;
    }
    srs_amd_dft* d = nullptr;
    if (srs_amd_dft_create(&d, config.size, config.dir == dft_processor::direction::DIRECT ? 0 : 1, dev) !=
        SRS_AMD_OK) {
      return nullptr;
    }
    return std::make_unique<dft_processor_hip>(d, config);
  }

private:
  int device;
};

} // namespace

std::shared_ptr<dft_processor_factory> srsran::hip::create_dft_processor_factory_hip(int device)
{
  return std::make_shared<dft_processor_factory_hip>(device);
}
