// perf_analyzer command line (flag spellings of the public perf_analyzer CLI,
// SURVEY.md Appendix D), plus a few MI355X extensions marked [ext].
#include <getopt.h>

#include <cstdlib>
#include <sstream>

#include "perf.h"

namespace tcperf {

namespace {

enum LongOnly {
  OPT_SYNC = 1000, OPT_ASYNC, OPT_STREAMING, OPT_SHAPE, OPT_CONC_RANGE, OPT_RATE_RANGE, OPT_DIST, OPT_INTERVALS,
  OPT_SEQ_LEN, OPT_SEQ_RANGE, OPT_INPUT_DATA, OPT_STR_LEN, OPT_STR_DATA, OPT_SHM, OPT_OUT_SHM_SIZE, OPT_MEAS_MODE,
  OPT_MEAS_COUNT, OPT_PERCENTILE, OPT_WARMUP, OPT_VERBOSE_CSV, OPT_JSON, OPT_RESUME, OPT_COLLECT_METRICS, OPT_METRICS_INTERVAL, OPT_METRICS_SYSFS, OPT_SHM_INPUT, OPT_SHM_OUTPUT, OPT_DEVICE, OPT_SEED,
  OPT_NUM_CLIENTS, OPT_NO_SERVER_STATS, OPT_GPUS, OPT_DEVICES, OPT_FANOUT, OPT_LOAD_PER_GPU, OPT_MEAS_INTERVAL, OPT_STABILITY, OPT_MAX_TRIALS, OPT_LAT_THRESH,
  OPT_SSL_GRPC_USE, OPT_SSL_GRPC_ROOT, OPT_SSL_GRPC_KEY, OPT_SSL_GRPC_CHAIN, OPT_SSL_HTTPS_PEER, OPT_SSL_HTTPS_HOST,
  OPT_SSL_HTTPS_CA, OPT_SSL_HTTPS_CERT, OPT_SSL_HTTPS_CERT_TYPE, OPT_SSL_HTTPS_KEY, OPT_SSL_HTTPS_KEY_TYPE,
  OPT_IN_FORMAT, OPT_OUT_FORMAT, OPT_GRPC_COMPRESSION, OPT_COMPRESSION, OPT_REQUEST_PARAM,
};

bool ParseU64(const std::string& s, uint64_t* v)
{
  if (s.empty()) return false;
  char* end = nullptr;
  unsigned long long x = strtoull(s.c_str(), &end, 10);
  if (*end != '\0') return false;
  *v = x;
  return true;
}

bool ParseDouble(const std::string& s, double* v)
{
  if (s.empty()) return false;
  char* end = nullptr;
  *v = strtod(s.c_str(), &end);
  return *end == '\0';
}

std::vector<std::string> Split(const std::string& s, char sep)
{
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

}  // namespace

std::string Usage()
{
  return
      "Usage: perf_analyzer -m <model> [options]\n"
      "  -m <model>                      model name (required)\n"
      "  -x <version>                     model version\n"
      "  -u <url>                         server URL (default localhost:8000 http / localhost:8001 grpc)\n"
      "  -i http|grpc                     protocol (default http)\n"
      "  -b <n>                           batch size (default 1)\n"
      "  -a, --async / --sync             asynchronous (default) or synchronous requests\n"
      "  --streaming                      use the gRPC bidirectional stream\n"
      "  --shape NAME:d1,d2,...           shape of a variable-size input (without batch dim)\n"
      "  -H 'Header:Value'                extra request header (repeatable)\n"
      "  --concurrency-range s[:e[:step]] closed-loop concurrency sweep (default 1)\n"
      "  --request-rate-range s[:e[:step]] open-loop request-rate sweep (requests/sec)\n"
      "  --request-distribution constant|poisson\n"
      "  --request-intervals <file>       open-loop inter-request intervals (usec per line)\n"
      "  --sequence-length <n>            requests per sequence for sequence models (default 20)\n"
      "  --sequence-id-range s[:e]        sequence ids to use\n"
      "  --input-data random|zero|<file.json>\n"
      "  --string-length <n> / --string-data <s>   BYTES synthetic data\n"
      "  --shared-memory none|system|cuda|hip      tensor transport (cuda is an alias of hip)\n"
      "  --output-shared-memory-size <bytes>       per-output region size (default 102400)\n"
      "  -p, --measurement-interval <ms>  time window (default 5000)\n"
      "  --measurement-mode time_windows|count_windows\n"
      "  --measurement-request-count <n>  requests per count window (default 50)\n"
      "  -s, --stability-percentage <pct> (default 10)\n"
      "  -r, --max-trials <n>             windows before giving up on stability (default 10)\n"
      "  --percentile <p>                 stabilise on and report pP latency instead of the average\n"
      "  -l, --latency-threshold <ms>     stop the sweep once latency exceeds this\n"
      "  --warmup-request-count <n>       requests before the first window\n"
      "  -f <file.csv>                    CSV report;  --verbose-csv adds per-point percentiles\n"
      "  -v                               verbose\n"
      "  [ext] --json-report <file>       machine-readable report (rewritten after every sweep point)\n"
      "  --collect-metrics                GPU utilization / power / VRAM of --device (amdgpu sysfs)\n"
      "  --metrics-interval <ms>          GPU metrics sampling interval (default 1000)\n"
      "  [ext] --resume                   skip sweep points already in --json-report (same model/batch/\n"
      "                                   protocol/shm/mode) and keep them in the reports\n"
      "  [ext] --shared-memory-input NAME=REGION[,REGION..]  use region(s) the caller already registered;\n"
      "                                   a list pins entry s % n to concurrency slot s\n"
      "  [ext] --shared-memory-output NAME=REGION[,REGION..]  caller output region(s), slot s -> s % n\n"
      "                                   (a list entry may be REGION@OFFSET: a slice of one region)\n"
      "  [ext] --device <gpu>             GPU for hip shared memory (default 0)\n"
      "  [ext] --seed <n>                 synthetic data seed (K1 Philox stream)\n"
      "  [ext] --num-clients <n>          protocol clients (connections) to spread requests over\n"
      "  [ext] --no-server-stats          skip ModelInferenceStatistics deltas\n"
      "  [ext] --gpus <n> | --devices a,b,c   multi-GPU load: one lane (client, worker thread, HIP stream,\n"
      "                                   shm regions) per GPU; per-GPU rows + an aggregate row\n"
      "  [ext] -u url0,url1,...           with several GPUs, lane i talks to url[i mod n]\n"
      "  [ext] --fanout rccl|p2p|host     how the synthetic batch made once on the first GPU reaches the\n"
      "                                   others (RCCL broadcast / xGMI peer-copy star / host copies)\n"
      "  [ext] --load-per-gpu             every GPU gets the full concurrency / rate (weak scaling);\n"
      "                                   default: the load is split over the GPUs\n"
      "  --input-tensor-format binary|json, --output-tensor-format binary|json\n"
      "                                   HTTP tensor encoding (json: inline \"data\" arrays)\n"
      "  --grpc-compression-algorithm none|gzip|deflate   gRPC message compression\n"
      "  [ext] --compression-algorithm none|gzip|deflate  the same for gRPC; for HTTP: request body and\n"
      "                                   response (Content-Encoding / Accept-Encoding)\n"
      "  --request-parameter name:value:type   custom request parameter (bool|int|string|double), repeatable\n"
      "  --ssl-grpc-use-ssl, --ssl-grpc-root-certifications-file F, --ssl-grpc-private-key-file F,\n"
      "  --ssl-grpc-certificate-chain-file F          gRPC over TLS (mutual TLS with key + chain)\n"
      "  --ssl-https-verify-peer 0|1, --ssl-https-verify-host 0|1|2, --ssl-https-ca-certificates-file F,\n"
      "  --ssl-https-client-certificate-file F, --ssl-https-client-certificate-type PEM|DER,\n"
      "  --ssl-https-private-key-file F, --ssl-https-private-key-type PEM|DER   HTTPS (https:// is implied)\n";
}

Error ParseOptions(int argc, char** argv, Options* o, bool* help)
{
  *help = false;
  static const struct option longopts[] = {
      {"model-name", required_argument, nullptr, 'm'},
      {"model-version", required_argument, nullptr, 'x'},
      {"url", required_argument, nullptr, 'u'},
      {"protocol", required_argument, nullptr, 'i'},
      {"batch-size", required_argument, nullptr, 'b'},
      {"async", no_argument, nullptr, OPT_ASYNC},
      {"sync", no_argument, nullptr, OPT_SYNC},
      {"streaming", no_argument, nullptr, OPT_STREAMING},
      {"shape", required_argument, nullptr, OPT_SHAPE},
      {"concurrency-range", required_argument, nullptr, OPT_CONC_RANGE},
      {"request-rate-range", required_argument, nullptr, OPT_RATE_RANGE},
      {"request-distribution", required_argument, nullptr, OPT_DIST},
      {"request-intervals", required_argument, nullptr, OPT_INTERVALS},
      {"sequence-length", required_argument, nullptr, OPT_SEQ_LEN},
      {"sequence-id-range", required_argument, nullptr, OPT_SEQ_RANGE},
      {"input-data", required_argument, nullptr, OPT_INPUT_DATA},
      {"string-length", required_argument, nullptr, OPT_STR_LEN},
      {"string-data", required_argument, nullptr, OPT_STR_DATA},
      {"shared-memory", required_argument, nullptr, OPT_SHM},
      {"output-shared-memory-size", required_argument, nullptr, OPT_OUT_SHM_SIZE},
      {"measurement-interval", required_argument, nullptr, OPT_MEAS_INTERVAL},
      {"measurement-mode", required_argument, nullptr, OPT_MEAS_MODE},
      {"measurement-request-count", required_argument, nullptr, OPT_MEAS_COUNT},
      {"stability-percentage", required_argument, nullptr, OPT_STABILITY},
      {"max-trials", required_argument, nullptr, OPT_MAX_TRIALS},
      {"percentile", required_argument, nullptr, OPT_PERCENTILE},
      {"latency-threshold", required_argument, nullptr, OPT_LAT_THRESH},
      {"warmup-request-count", required_argument, nullptr, OPT_WARMUP},
      {"verbose-csv", no_argument, nullptr, OPT_VERBOSE_CSV},
      {"json-report", required_argument, nullptr, OPT_JSON},
      {"resume", no_argument, nullptr, OPT_RESUME},
      {"collect-metrics", no_argument, nullptr, OPT_COLLECT_METRICS},
      {"metrics-interval", required_argument, nullptr, OPT_METRICS_INTERVAL},
      {"metrics-sysfs-root", required_argument, nullptr, OPT_METRICS_SYSFS},
      {"shared-memory-input", required_argument, nullptr, OPT_SHM_INPUT},
      {"shared-memory-output", required_argument, nullptr, OPT_SHM_OUTPUT},
      {"device", required_argument, nullptr, OPT_DEVICE},
      {"seed", required_argument, nullptr, OPT_SEED},
      {"num-clients", required_argument, nullptr, OPT_NUM_CLIENTS},
      {"no-server-stats", no_argument, nullptr, OPT_NO_SERVER_STATS},
      {"gpus", required_argument, nullptr, OPT_GPUS},
      {"devices", required_argument, nullptr, OPT_DEVICES},
      {"fanout", required_argument, nullptr, OPT_FANOUT},
      {"load-per-gpu", no_argument, nullptr, OPT_LOAD_PER_GPU},
      {"ssl-grpc-use-ssl", no_argument, nullptr, OPT_SSL_GRPC_USE},
      {"ssl-grpc-root-certifications-file", required_argument, nullptr, OPT_SSL_GRPC_ROOT},
      {"ssl-grpc-private-key-file", required_argument, nullptr, OPT_SSL_GRPC_KEY},
      {"ssl-grpc-certificate-chain-file", required_argument, nullptr, OPT_SSL_GRPC_CHAIN},
      {"ssl-https-verify-peer", required_argument, nullptr, OPT_SSL_HTTPS_PEER},
      {"ssl-https-verify-host", required_argument, nullptr, OPT_SSL_HTTPS_HOST},
      {"ssl-https-ca-certificates-file", required_argument, nullptr, OPT_SSL_HTTPS_CA},
      {"ssl-https-client-certificate-file", required_argument, nullptr, OPT_SSL_HTTPS_CERT},
      {"ssl-https-client-certificate-type", required_argument, nullptr, OPT_SSL_HTTPS_CERT_TYPE},
      {"ssl-https-private-key-file", required_argument, nullptr, OPT_SSL_HTTPS_KEY},
      {"ssl-https-private-key-type", required_argument, nullptr, OPT_SSL_HTTPS_KEY_TYPE},
      {"input-tensor-format", required_argument, nullptr, OPT_IN_FORMAT},
      {"output-tensor-format", required_argument, nullptr, OPT_OUT_FORMAT},
      {"grpc-compression-algorithm", required_argument, nullptr, OPT_GRPC_COMPRESSION},
      {"compression-algorithm", required_argument, nullptr, OPT_COMPRESSION},
      {"request-parameter", required_argument, nullptr, OPT_REQUEST_PARAM},
      {"verbose", no_argument, nullptr, 'v'},
      {"help", no_argument, nullptr, 'h'},
      {nullptr, 0, nullptr, 0}};
  optind = 1;
  opterr = 0;
  int c;
  uint64_t u = 0;
  double d = 0;
  while ((c = getopt_long(argc, argv, "m:x:u:i:b:aH:p:s:r:l:f:t:vh", longopts, nullptr)) != -1) {
    const std::string arg = optarg ? optarg : "";
    switch (c) {
      case 'm': o->model = arg; break;
      case 'x': o->version = arg; break;
      case 'u': o->url = arg; break;
      case 'i':
        if (arg != "http" && arg != "grpc" && arg != "HTTP" && arg != "gRPC" && arg != "GRPC")
          return Error("-i expects http or grpc, got '" + arg + "'");
        o->protocol = (arg == "http" || arg == "HTTP") ? "http" : "grpc";
        break;
      case 'b':
        if (!ParseU64(arg, &u) || u == 0) return Error("-b expects a positive integer");
        o->batch = static_cast<int>(u);
        break;
      case 'a': case OPT_ASYNC: o->async = true; break;
      case OPT_SYNC: o->async = false; break;
      case OPT_STREAMING: o->streaming = true; break;
      case 'H': {
        auto p = arg.find(':');
        if (p == std::string::npos) return Error("-H expects 'Name:Value'");
        o->headers[arg.substr(0, p)] = arg.substr(p + 1);
        break;
      }
      case OPT_SHAPE: {
        auto p = arg.rfind(':');
        if (p == std::string::npos) return Error("--shape expects NAME:d1,d2,...");
        std::vector<int64_t> dims;
        for (const auto& t : Split(arg.substr(p + 1), ',')) {
          if (!ParseU64(t, &u)) return Error("bad --shape dims '" + arg + "'");
          dims.push_back(static_cast<int64_t>(u));
        }
        o->shapes[arg.substr(0, p)] = dims;
        break;
      }
      case 't':
      case OPT_CONC_RANGE: {
        auto parts = Split(arg, ':');
        if (parts.size() > 3 || !ParseU64(parts[0], &o->conc_start)) return Error("bad --concurrency-range");
        o->conc_end = o->conc_start;
        o->conc_step = 1;
        if (parts.size() > 1 && !ParseU64(parts[1], &o->conc_end)) return Error("bad --concurrency-range");
        if (parts.size() > 2 && (!ParseU64(parts[2], &o->conc_step) || o->conc_step == 0))
          return Error("bad --concurrency-range");
        if (o->conc_end < o->conc_start) return Error("--concurrency-range end < start");
        o->rate_mode = false;
        break;
      }
      case OPT_RATE_RANGE: {
        auto parts = Split(arg, ':');
        if (parts.size() > 3 || !ParseDouble(parts[0], &o->rate_start) || o->rate_start <= 0)
          return Error("bad --request-rate-range");
        o->rate_end = o->rate_start;
        o->rate_step = 1;
        if (parts.size() > 1 && !ParseDouble(parts[1], &o->rate_end)) return Error("bad --request-rate-range");
        if (parts.size() > 2 && (!ParseDouble(parts[2], &o->rate_step) || o->rate_step <= 0))
          return Error("bad --request-rate-range");
        o->rate_mode = true;
        break;
      }
      case OPT_DIST:
        if (arg != "constant" && arg != "poisson") return Error("--request-distribution: constant|poisson");
        o->distribution = arg;
        break;
      case OPT_INTERVALS: o->request_intervals_file = arg; o->rate_mode = true; break;
      case OPT_SEQ_LEN:
        if (!ParseU64(arg, &u) || u == 0) return Error("bad --sequence-length");
        o->sequence_length = static_cast<int>(u);
        break;
      case OPT_SEQ_RANGE: {
        auto parts = Split(arg, ':');
        if (!ParseU64(parts[0], &o->seq_id_start)) return Error("bad --sequence-id-range");
        if (parts.size() > 1 && !ParseU64(parts[1], &o->seq_id_end)) return Error("bad --sequence-id-range");
        if (o->seq_id_end <= o->seq_id_start) return Error("--sequence-id-range end must be > start");
        break;
      }
      case OPT_INPUT_DATA: o->input_data = arg; break;
      case OPT_STR_LEN:
        if (!ParseU64(arg, &u)) return Error("bad --string-length");
        o->string_length = static_cast<int>(u);
        break;
      case OPT_STR_DATA: o->string_data = arg; break;
      case OPT_SHM:
        if (arg != "none" && arg != "system" && arg != "cuda" && arg != "hip")
          return Error("--shared-memory: none|system|cuda|hip");
        o->shared_memory = (arg == "cuda") ? "hip" : arg;
        break;
      case OPT_OUT_SHM_SIZE:
        if (!ParseU64(arg, &u)) return Error("bad --output-shared-memory-size");
        o->output_shm_size = u;
        break;
      case 'p': case OPT_MEAS_INTERVAL:
        if (!ParseU64(arg, &o->measurement_interval_ms) || o->measurement_interval_ms == 0)
          return Error("bad --measurement-interval");
        break;
      case OPT_MEAS_MODE:
        if (arg != "time_windows" && arg != "count_windows")
          return Error("--measurement-mode: time_windows|count_windows");
        o->measurement_mode = arg;
        break;
      case OPT_MEAS_COUNT:
        if (!ParseU64(arg, &o->measurement_request_count) || o->measurement_request_count == 0)
          return Error("bad --measurement-request-count");
        break;
      case 's': case OPT_STABILITY:
        if (!ParseDouble(arg, &d) || d <= 0) return Error("bad --stability-percentage");
        o->stability_pct = d;
        break;
      case 'r': case OPT_MAX_TRIALS:
        if (!ParseU64(arg, &u) || u == 0) return Error("bad --max-trials");
        o->max_trials = static_cast<int>(u);
        break;
      case OPT_PERCENTILE:
        if (!ParseU64(arg, &u) || u == 0 || u > 99) return Error("--percentile expects 1..99");
        o->percentile = static_cast<int>(u);
        break;
      case 'l': case OPT_LAT_THRESH:
        if (!ParseU64(arg, &o->latency_threshold_ms)) return Error("bad --latency-threshold");
        break;
      case OPT_WARMUP:
        if (!ParseU64(arg, &o->warmup_requests)) return Error("bad --warmup-request-count");
        break;
      case 'f': o->csv_file = arg; break;
      case OPT_VERBOSE_CSV: o->verbose_csv = true; break;
      case OPT_JSON: o->json_file = arg; break;
      case OPT_RESUME: o->resume = true; break;
      case OPT_COLLECT_METRICS: o->collect_metrics = true; break;
      case OPT_METRICS_INTERVAL: o->metrics_interval_ms = std::stoull(arg); break;
      case OPT_METRICS_SYSFS: o->metrics_sysfs_root = arg; break;
      case OPT_SHM_INPUT: {
        auto p = arg.find('=');
        if (p == std::string::npos) return Error("--shared-memory-input expects NAME=REGION");
        const std::string name = arg.substr(0, p), val = arg.substr(p + 1);
        if (val.find(',') == std::string::npos) {
          o->preregistered_inputs[name] = val;
        } else {
          auto& l = o->preregistered_input_lists[name];
          for (size_t b = 0; b <= val.size();) {
            size_t c = val.find(',', b);
            if (c == std::string::npos) c = val.size();
            if (c > b) l.push_back(val.substr(b, c - b));
            b = c + 1;
          }
          if (l.empty()) return Error("--shared-memory-input: no region for " + name);
          o->preregistered_inputs[name] = l.front();
        }
        break;
      }
      case OPT_SHM_OUTPUT: {
        auto p = arg.find('=');
        if (p == std::string::npos) return Error("--shared-memory-output expects NAME=REGION[,REGION..]");
        const std::string val = arg.substr(p + 1);
        auto& l = o->preregistered_outputs[arg.substr(0, p)];
        for (size_t b = 0; b <= val.size();) {
          size_t c = val.find(',', b);
          if (c == std::string::npos) c = val.size();
          if (c > b) l.push_back(val.substr(b, c - b));
          b = c + 1;
        }
        if (l.empty()) return Error("--shared-memory-output: no region for " + arg.substr(0, p));
        break;
      }
      case OPT_DEVICE:
        if (!ParseU64(arg, &u)) return Error("bad --device");
        o->device = static_cast<int>(u);
        break;
      case OPT_SEED:
        if (!ParseU64(arg, &o->seed)) return Error("bad --seed");
        break;
      case OPT_NUM_CLIENTS:
        if (!ParseU64(arg, &u)) return Error("bad --num-clients");
        o->num_clients = static_cast<int>(u);
        break;
      case OPT_NO_SERVER_STATS: o->collect_server_stats = false; break;
      case OPT_GPUS:
        if (!ParseU64(arg, &u) || u == 0 || u > 64) return Error("bad --gpus (1..64)");
        o->devices.clear();
        for (uint64_t d = 0; d < u; ++d) o->devices.push_back(static_cast<int>(d));
        break;
      case OPT_DEVICES: {
        o->devices.clear();
        std::stringstream ss(arg);
        std::string tok;
        while (std::getline(ss, tok, ',')) {
          if (!ParseU64(tok, &u) || u > 63) return Error("bad --devices entry '" + tok + "'");
          o->devices.push_back(static_cast<int>(u));
        }
        if (o->devices.empty()) return Error("--devices needs at least one GPU");
        break;
      }
      case OPT_FANOUT:
        if (arg != "rccl" && arg != "p2p" && arg != "host" && arg != "auto") return Error("--fanout: rccl|p2p|host");
        o->fanout = arg;
        break;
      case OPT_LOAD_PER_GPU: o->load_per_gpu = true; break;
      case OPT_SSL_GRPC_USE: o->ssl.grpc_use_ssl = true; break;
      case OPT_SSL_GRPC_ROOT: o->ssl.grpc_root_certs = arg; o->ssl.grpc_use_ssl = true; break;
      case OPT_SSL_GRPC_KEY: o->ssl.grpc_private_key = arg; o->ssl.grpc_use_ssl = true; break;
      case OPT_SSL_GRPC_CHAIN: o->ssl.grpc_cert_chain = arg; o->ssl.grpc_use_ssl = true; break;
      case OPT_SSL_HTTPS_PEER:
        if (!ParseU64(arg, &u) || u > 1) return Error("--ssl-https-verify-peer expects 0 or 1");
        o->ssl.https_verify_peer = static_cast<long>(u);
        o->ssl.https = true;
        break;
      case OPT_SSL_HTTPS_HOST:
        if (!ParseU64(arg, &u) || u > 2) return Error("--ssl-https-verify-host expects 0, 1 or 2");
        o->ssl.https_verify_host = static_cast<long>(u);
        o->ssl.https = true;
        break;
      case OPT_SSL_HTTPS_CA: o->ssl.https_ca = arg; o->ssl.https = true; break;
      case OPT_SSL_HTTPS_CERT: o->ssl.https_cert = arg; o->ssl.https = true; break;
      case OPT_SSL_HTTPS_KEY: o->ssl.https_key = arg; o->ssl.https = true; break;
      case OPT_SSL_HTTPS_CERT_TYPE:
      case OPT_SSL_HTTPS_KEY_TYPE:
        if (arg != "PEM" && arg != "DER") return Error("certificate / key type must be PEM or DER");
        (c == OPT_SSL_HTTPS_CERT_TYPE ? o->ssl.https_cert_der : o->ssl.https_key_der) = arg == "DER";
        o->ssl.https = true;
        break;
      case OPT_IN_FORMAT:
      case OPT_OUT_FORMAT:
        if (arg != "binary" && arg != "json") return Error("tensor formats are binary or json, got '" + arg + "'");
        (c == OPT_IN_FORMAT ? o->input_tensor_format : o->output_tensor_format) = arg;
        break;
      case OPT_GRPC_COMPRESSION:
      case OPT_COMPRESSION:
        if (arg != "none" && arg != "gzip" && arg != "deflate")
          return Error("compression algorithms are none, gzip or deflate, got '" + arg + "'");
        o->compression = arg;
        break;
      case OPT_REQUEST_PARAM: {
        // name:value:type, type one of bool|int|string|double (value may contain ':')
        const size_t a = arg.find(':'), b = arg.rfind(':');
        if (a == std::string::npos || a == b || a == 0) return Error("--request-parameter expects name:value:type");
        triton::client::RequestParameter rp;
        rp.name = arg.substr(0, a);
        rp.value = arg.substr(a + 1, b - a - 1);
        rp.type = arg.substr(b + 1);
        if (rp.type != "bool" && rp.type != "int" && rp.type != "string" && rp.type != "double")
          return Error("--request-parameter type must be bool, int, string or double, got '" + rp.type + "'");
        if (rp.type == "bool" && rp.value != "true" && rp.value != "false")
          return Error("--request-parameter bool values are true or false");
        if (rp.type == "int") {
          char* end = nullptr;
          strtoll(rp.value.c_str(), &end, 10);
          if (rp.value.empty() || *end) return Error("--request-parameter: bad int '" + rp.value + "'");
        }
        if (rp.type == "double") {
          char* end = nullptr;
          strtod(rp.value.c_str(), &end);
          if (rp.value.empty() || *end) return Error("--request-parameter: bad double '" + rp.value + "'");
        }
        o->request_parameters[rp.name] = rp;
        break;
      }
      case 'v': o->verbose = true; break;
      case 'h': *help = true; return Error::Success;
      default: {
        std::string bad = (optind - 1 < argc && optind >= 1) ? argv[optind - 1] : "?";
        return Error("unknown or incomplete option '" + bad + "'");
      }
    }
  }
  if (optind < argc) return Error(std::string("unexpected argument '") + argv[optind] + "'");
  if (o->model.empty()) return Error("-m <model> is required");
  if (o->url.empty()) o->url = o->protocol == "grpc" ? "localhost:8001" : "localhost:8000";
  {
    std::stringstream ss(o->url);
    std::string tok;
    o->urls.clear();
    while (std::getline(ss, tok, ','))
      if (!tok.empty()) o->urls.push_back(tok);
    if (o->urls.empty()) return Error("bad -u");
    o->url = o->urls[0];
  }
  if (o->devices.empty()) o->devices.push_back(o->device);
  o->device = o->devices[0];
  if (o->urls.size() > 1 && o->urls.size() != o->devices.size())
    return Error("-u lists " + std::to_string(o->urls.size()) + " URLs for " + std::to_string(o->devices.size()) +
                 " GPUs (give one URL, or one per GPU)");
  if (o->streaming && o->protocol != "grpc") return Error("--streaming requires -i grpc");
  if ((o->input_tensor_format == "json" || o->output_tensor_format == "json") && o->protocol != "http")
    return Error("--input-tensor-format / --output-tensor-format json need -i http");
  if (!o->preregistered_inputs.empty() && o->shared_memory == "none")
    return Error("--shared-memory-input requires --shared-memory system|hip");
  if (!o->preregistered_outputs.empty() && o->shared_memory == "none")
    return Error("--shared-memory-output requires --shared-memory system|hip");
  if (!o->preregistered_input_lists.empty() && o->input_data != "random" && o->input_data != "zero")
    return Error("--shared-memory-input region lists and JSON --input-data are exclusive");
  return Error::Success;
}

}  // namespace tcperf
