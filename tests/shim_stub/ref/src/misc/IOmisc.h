// Stand-in for the reference's src/misc/IOmisc.h: the report stream BA logs to.
#pragma once
#include <fstream>
struct LogFilesStreams {
    std::fstream mainReportStream;
};
extern LogFilesStreams logStreams;
