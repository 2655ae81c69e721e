// Stand-in for the reference's src/config/config.h + ConfigService.h +
// configData.h: the fields the shim reads and the getValue<T> accessor.
#pragma once
enum ConfigFieldEnum {
    FM_KNN_DISTANCE,
    BA_USE_TRIVIAL_LOSS, BA_USE_HUBER_LOSS, BA_HUBER_LOSS_PARAMETER, BA_USE_CAUCHY_LOSS, BA_CAUCHY_LOSS_PARAMETER,
    BA_USE_ARCTAN_LOSS, BA_ARCTAN_LOSS_PARAMETER, BA_USE_TUKEY_LOSS, BA_TUKEY_LOSS_PARAMETER
};
class ConfigService {
public:
    template <typename T> T getValue(ConfigFieldEnum enumKey);
};
extern ConfigService configService;
