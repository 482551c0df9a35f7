// ldpc_decoder_hip.cpp -- srsran::ldpc_decoder over srs_amd_ldpc_decode (see the header).
#include "ldpc_decoder_hip.h"

#include "srsran/adt/bit_buffer.h"
#include "srsran_amd/ldpc.h"

#include <cstdio>

using namespace srsran;

namespace {

class ldpc_decoder_hip : public ldpc_decoder
{
public:
  explicit ldpc_decoder_hip(srs_amd_ldpc_decoder* dec_) : dec(dec_) {}
  ~ldpc_decoder_hip() override { srs_amd_ldpc_decoder_destroy(dec); }

  // ldpc_decoder_impl.cpp:55 semantics: trimmed input, CRC early stop, nullopt without a CRC pass (or always
  // nullopt without a CRC calculator, as the reference returns after max_iterations).  A failed decode (an invalid
  // configuration the reference would assert on, or a HIP runtime error) is logged and reported as "no CRC pass":
  // the gNB keeps running and the codeblock counts as failed (HARQ retransmission).
  std::optional<unsigned> decode(bit_buffer&                      output,
                                 span<const log_likelihood_ratio> input,
                                 crc_calculator*                  crc,
                                 const configuration&             cfg) override
  {
    const srs_amd_ldpc_decoder_config c = {cfg.base_graph == ldpc_base_graph_type::BG1 ? 1u : 2u,
                                           static_cast<uint32_t>(cfg.lifting_size), cfg.nof_filler_bits,
                                           cfg.nof_crc_bits, cfg.max_iterations};
    int32_t   iters = -1;
    const int rc    = srs_amd_ldpc_decode(dec, output.get_buffer().data(),
                                       reinterpret_cast<const int8_t*>(input.data()), input.size(),
                                       crc ? static_cast<int>(crc->get_generator_poly()) : SRS_AMD_NO_CRC, &c, &iters);
    if (rc != SRS_AMD_OK) {
      std::fprintf(stderr, "ldpc_decoder_hip: decode failed (reported as a CRC failure): %s\n", srs_amd_last_error());
      return std::nullopt;
    }
    if (iters < 0) {
      return std::nullopt;
    }
    return static_cast<unsigned>(iters);
  }

private:
  srs_amd_ldpc_decoder* dec = nullptr;
};

class ldpc_decoder_factory_hip : public ldpc_decoder_factory
{
public:
  ldpc_decoder_factory_hip(int arith_, bool force_, int device_) : arith(arith_), force(force_), device(device_) {}
  // nullptr when the decoder cannot be created (no device, out of memory), as the reference's factories report a
  // creation failure; the error is logged.
  std::unique_ptr<ldpc_decoder> create() override
  {
    srs_amd_ldpc_decoder* dec = nullptr;
    if (srs_amd_ldpc_decoder_create(&dec, arith, force ? 1 : 0, device) != SRS_AMD_OK) {
      std::fprintf(stderr, "ldpc_decoder_hip: decoder creation failed: %s\n", srs_amd_last_error());
      return nullptr;
    }
    return std::make_unique<ldpc_decoder_hip>(dec);
  }

private:
  int  arith;
  bool force;
  int  device;
};

} // namespace

std::shared_ptr<ldpc_decoder_factory>
srsran::hip::create_ldpc_decoder_factory_hip(const std::string& dec_type, bool force_decoding, int device)
{
  if (dec_type == "hip") {
    return std::make_shared<ldpc_decoder_factory_hip>(SRS_AMD_ARITH_SIMD, force_decoding, device);
  }
  if (dec_type == "hip-generic") {
    return std::make_shared<ldpc_decoder_factory_hip>(SRS_AMD_ARITH_GENERIC, force_decoding, device);
  }
  return nullptr;
}
