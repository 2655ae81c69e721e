"""The reference's JSON configuration surface (src/config/*).

Same 40 keys and types as configData.h:73-126, same strictness as
ConfigService::checkJSON (config.cpp:23-51): every key must be present with a
compatible type, otherwise the reference prints "Field ... missed or has
incorrect type!" and exit(2)s -- here ConfigError is raised with the same text
(and a CLI shim can turn it into exit code 2).  Comments are accepted as in
json::parse(stream, nullptr, true, /*ignore_comments*/ true) (config.cpp:13).

Keys this build adds are OPTIONAL so that every reference config still loads:
  gpuCount (int, default: all visible GPUs) -- candidate sharding width.
"""
import json

BOOL, STRING, INTEGER, FLOATING = "BOOLEAN", "STRING", "INTEGER", "FLOATING POINT NUMBER"

# configData.h:73-126, in declaration order
CONFIG_FIELDS = [
    ("onlyViz", BOOL), ("calibrate", BOOL), ("visualCalibration", BOOL), ("calibrationPath", STRING),
    ("usePhotosCycle", BOOL), ("photosPathPattern", STRING), ("videoSourcePath", STRING),
    ("outputDataDir", STRING), ("threadsCount", INTEGER), ("useUndistortion", BOOL),
    ("requiredExtractedPointsCount", INTEGER), ("featureExtractingThreshold", INTEGER),
    ("framesBatchSize", INTEGER), ("skipFramesFromBatchHead", INTEGER), ("useFirstFitInBatch", BOOL),
    ("requiredMatchedPointsCount", INTEGER), ("useFM-SIFT-FLANN", BOOL), ("useFM-SIFT-BF", BOOL),
    ("useFM-ORB", BOOL), ("knnMatcherDistance", FLOATING), ("RPUseRANSAC", BOOL), ("RPRANSACProb", FLOATING),
    ("RPRANSACThreshold", FLOATING), ("RPDistanceThreshold", FLOATING), ("useBundleAdjustment", BOOL),
    ("BAMaxFramesCnt", INTEGER), ("BAThreadsCnt", INTEGER), ("BAUseTrivialLossFunction", BOOL),
    ("BAUseHuberLossFunction", BOOL), ("BAHuberLossFunctionParameter", FLOATING),
    ("BAUseCauchyLossFunction", BOOL), ("BACauchyLossFunctionParameter", FLOATING),
    ("BAUseArctanLossFunction", BOOL), ("BAArctanLossFunctionParameter", FLOATING),
    ("BAUseTukeyLossFunction", BOOL), ("BATukeyLossFunctionParameter", FLOATING),
    ("TriangleMaxDistance", FLOATING), ("TriangleEuclidDistanceWeight", FLOATING),
    ("TriangleColorDistance", FLOATING), ("TriangleMinimumPoints", INTEGER),
]
OPTIONAL_FIELDS = {"gpuCount": INTEGER}


class ConfigError(ValueError):
    """checkJSON / setConfigFile failure (the reference exit(2)s)."""


def strip_comments(text):
    """Remove // and /* */ comments outside string literals."""
    out, i, n, in_str = [], 0, len(text), False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 2
                continue
            if c == '"':
                in_str = False
            i += 1
        elif c == '"':
            in_str = True
            out.append(c)
            i += 1
        elif text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            if j < 0:
                raise ConfigError("Failed to parse JSON config")
            i = j + 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _type_ok(value, kind):
    # nlohmann get<T>: bool needs a boolean; numbers accept int/float/bool;
    # strings need a string; a missing key reads as null and fails every type.
    if kind == BOOL:
        return isinstance(value, bool)
    if kind in (INTEGER, FLOATING):
        return isinstance(value, (int, float))
    return isinstance(value, str)


class ConfigService:
    """Mirror of src/config/ConfigService.h."""

    def __init__(self, data=None):
        self.config = {} if data is None else dict(data)

    def setConfigFile(self, path):
        try:
            with open(path, encoding="utf-8") as f:
                text = f.read()
        except OSError as e:
            raise ConfigError("Failed to open config file") from e
        self.setConfigText(text)

    def setConfigText(self, text):
        try:
            self.config = json.loads(strip_comments(text))
        except (json.JSONDecodeError, ConfigError) as e:
            raise ConfigError("Failed to parse JSON config\n"
                              "Make sure you specified path to JSON with correct semantics") from e
        self.checkJSON()

    def checkJSON(self):
        for key, kind in CONFIG_FIELDS:
            if key not in self.config or not _type_ok(self.config[key], kind):
                raise ConfigError(f'Field "{key}" missed or has incorrect type!\nCorrect type is {kind}')
        for key, kind in OPTIONAL_FIELDS.items():
            if key in self.config and not _type_ok(self.config[key], kind):
                raise ConfigError(f'Field "{key}" missed or has incorrect type!\nCorrect type is {kind}')

    def getValue(self, key, kind=None):
        v = self.config[key]
        if kind == INTEGER and isinstance(v, (int, float)):
            return int(v)
        if kind == FLOATING:
            return float(v)
        return v

    def get(self, key, default=None):
        return self.config.get(key, default)


def reference_example():
    """The README.md:142-207 example config with the 4 Triangle* keys it lacks
    (configData.h:122-125) -- a complete, valid configuration."""
    return {
        "onlyViz": False, "calibrate": False, "visualCalibration": True,
        "calibrationPath": "./config/samsung-hv.xml", "usePhotosCycle": False,
        "photosPathPattern": "", "videoSourcePath": "", "outputDataDir": "./data",
        "threadsCount": 1, "useUndistortion": False, "requiredExtractedPointsCount": 10000,
        "featureExtractingThreshold": 1, "framesBatchSize": 210, "skipFramesFromBatchHead": 0,
        "useFirstFitInBatch": True, "requiredMatchedPointsCount": 500, "useFM-SIFT-FLANN": True,
        "useFM-SIFT-BF": False, "useFM-ORB": False, "knnMatcherDistance": 0.7, "RPUseRANSAC": True,
        "RPRANSACProb": 0.999, "RPRANSACThreshold": 5.0, "RPDistanceThreshold": 200.0,
        "useBundleAdjustment": False, "BAMaxFramesCnt": 8, "BAThreadsCnt": 12,
        "BAUseTrivialLossFunction": False, "BAUseHuberLossFunction": True,
        "BAHuberLossFunctionParameter": 4.0, "BAUseCauchyLossFunction": False,
        "BACauchyLossFunctionParameter": 4.0, "BAUseArctanLossFunction": False,
        "BAArctanLossFunctionParameter": 2.0, "BAUseTukeyLossFunction": False,
        "BATukeyLossFunctionParameter": 4.0, "TriangleMaxDistance": 1.0,
        "TriangleEuclidDistanceWeight": 1.0, "TriangleColorDistance": 1.0, "TriangleMinimumPoints": 3,
    }
