// generic.hip — the generic device-interpreter back ends (dae_device.hpp),
// one per size class; selected when no generated back end matches a model.
#include "core.hpp"

const Backend* generic_backends() {
    static const Backend kGeneric[4] = {
        make_backend_lane<GenericDae<SzSmall>>("generic-small", 0.0),
        make_backend_lane<GenericDae<SzMedium>>("generic-medium", 0.0),
        make_backend_lane<GenericDae<SzLarge>>("generic-large", 0.0),
        make_backend_lane<GenericDae<SzBody>>("generic-body", 0.0),
    };
    return kGeneric;
}
