"""srsran_project_amd -- MI355X-native (gfx950 HIP) implementation of srsRAN's
PUSCH/PDSCH channel-coding hot path behind the reference's own interfaces.

See DESIGN.md for the path, the boundary and the kernels.
"""
from . import _lib  # noqa: F401
from .ldpc import (  # noqa: F401
    CrcGeneratorPoly,
    LdpcBaseGraph,
    LdpcDecoder,
    LdpcDecoderConfiguration,
    LdpcDecoderFactory,
    LIFTING_SIZES,
    codeblock_length,
    create_ldpc_decoder_factory_hip,
    message_length,
)

from .ldpc_codec import (  # noqa: F401
    CodeblockMetadata,
    LdpcEncoder,
    LdpcEncoderConfiguration,
    LdpcRateDematcher,
    LdpcRateMatcher,
    MODULATION_ORDER,
    create_ldpc_encoder_factory_hip,
    create_ldpc_rate_dematcher_factory_hip,
    create_ldpc_rate_matcher_factory_hip,
)

from .ofdm import (  # noqa: F401
    CyclicPrefix,
    DftDirection,
    DftProcessor,
    OfdmDemodulatorConfiguration,
    OfdmModulatorConfiguration,
    OfdmSlotDemodulator,
    OfdmSlotModulator,
    create_dft_processor_factory_hip,
    create_ofdm_demodulator_factory_hip,
    create_ofdm_modulator_factory_hip,
)

from .equalizer import (  # noqa: F401
    ChannelEqualizer,
    ChannelEqualizerAlgorithmType,
    create_channel_equalizer_generic_factory_hip,
)

from .polar import (  # noqa: F401
    PolarCode,
    PolarCodeIbil,
    PolarInterleaverDirection,
    polar_code_construct,
    polar_interleave,
)

from .modulation import MODULATION, Modulator  # noqa: F401

from .crc import CrcCalculator, create_crc_calculator_factory_hip  # noqa: F401

from .pdsch_modulator import (  # noqa: F401
    DmrsPdschConfig,
    PdschModPlan,
    PdschModulator,
    PdschModulatorConfig,
    PdschSlot,
    PdschSlotPdu,
    ReservedPattern,
)

from .pusch_chest import (  # noqa: F401
    ChestPortStats,
    DmrsPuschEstimator,
    DmrsPuschEstimatorConfig,
    FdSmoothingStrategy,
    TdInterpolationStrategy,
    low_papr_length_valid,
    low_papr_sequence,
)

from .pusch_demodulator import PuschDemodPlan, PuschDemodulator, PuschDemodulatorConfig  # noqa: F401

from .pusch_processor import (  # noqa: F401
    PuschPdu,
    PuschProcessor,
    PuschProcessorConfig,
    PuschSlot,
    PuschSlotPdu,
    PuschSlotIo,
    PuschProcessorPlan,
    PuschProcessorResult,
    UciPart2SizeDescription,
    make_pdu,
    uci_part2_description,
    uci_part2_get_size,
)

from .sch import (  # noqa: F401
    PdschEncoder,
    PdschUe,
    PuschDecoder,
    PuschDecoderConfig,
    PuschDecoderResult,
    PuschUe,
    SchPlan,
    SlotUes,
    sch_plan,
    sch_segments,
    soft_buffer_size,
    decoder_llr_prefix,
    tbs_calculator_calculate,
)
__version__ = "0.1.0"

from .transform_precoding import TransformPrecoder, is_nof_prbs_valid as transform_precoding_nof_prbs_valid  # noqa: F401,E402

from .ulsch_info import UlschConfig, UlschInfo, ulsch_information  # noqa: F401,E402
from .ulsch_demux import UlschDemux, UlschDemuxConfig, UlschDemuxPlan  # noqa: F401,E402
from .uci_decoder import UCI_INVALID, UCI_UNKNOWN, UCI_VALID, UciDecoder  # noqa: F401,E402
from . import profiling  # noqa: F401,E402
from . import pdcch  # noqa: F401,E402
from .pdcch import CceToRegMapping, PdcchPdu, PdcchProcessor  # noqa: F401,E402
from . import ssb  # noqa: F401,E402
from .ssb import SsbPatternCase, SsbPdu, SsbProcessor  # noqa: F401,E402
from . import pucch  # noqa: F401,E402
from .pucch import PucchF0Pdu, PucchF1Batch, PucchF2Pdu, PucchF34Pdu, PucchProcessor  # noqa: F401,E402
