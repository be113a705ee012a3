#!/bin/bash
# Java bindings of the native C APIs this framework exposes, via javacpp
# (reference src/java-api-bindings/scripts/install_dependencies_and_build.sh,
# which binds the Triton server C API the same way).
#
#   libtcserve.so      native gRPC front end (csrc/cpp/server/tcserve.h)
#   libperfanalyzer.so perf engine C ABI      (csrc/cpp/perf/capi.cc)
#
# Needs a JDK, maven and network access for javacpp (not available in the
# build image).  Usage: install_dependencies_and_build.sh [--javacpp-version X]
set -euo pipefail
JAVACPP_VERSION=1.5.9
while [[ $# -gt 0 ]]; do
  case "$1" in
    --javacpp-version) JAVACPP_VERSION="$2"; shift 2 ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
done
HERE="$(cd "$(dirname "$0")/.." && pwd)"
REPO="$(cd "${HERE}/../.." && pwd)"
for tool in javac mvn make; do
  command -v "$tool" > /dev/null || { echo "missing $tool" >&2; exit 1; }
done

# 1. native libraries
make -C "${REPO}/csrc/cpp" -j"${MAX_JOBS:-8}" build/lib/libtcserve.so build/lib/libperfanalyzer.so

# 2. javacpp presets project
WORK="${HERE}/build"
mkdir -p "${WORK}/src/main/java/triton/amd/presets"
cat > "${WORK}/src/main/java/triton/amd/presets/tcnative.java" <<JAVA
package triton.amd.presets;

import org.bytedeco.javacpp.annotation.*;
import org.bytedeco.javacpp.tools.*;

@Properties(target = "triton.amd.tcnative", value = @Platform(
    include = {"tcserve.h"},
    includepath = {"${REPO}/csrc/cpp/server"},
    link = {"tcserve", "perfanalyzer"},
    linkpath = {"${REPO}/csrc/cpp/build/lib"}))
public class tcnative implements InfoMapper {
  public void map(InfoMap infoMap) {}
}
JAVA
cat > "${WORK}/pom.xml" <<POM
<project xmlns="http://maven.apache.org/POM/4.0.0">
  <modelVersion>4.0.0</modelVersion>
  <groupId>triton.amd</groupId>
  <artifactId>tcnative</artifactId>
  <version>0.1.0</version>
  <properties><maven.compiler.release>11</maven.compiler.release></properties>
  <dependencies>
    <dependency><groupId>org.bytedeco</groupId><artifactId>javacpp</artifactId><version>${JAVACPP_VERSION}</version></dependency>
  </dependencies>
  <build><plugins><plugin>
    <groupId>org.bytedeco</groupId><artifactId>javacpp</artifactId><version>${JAVACPP_VERSION}</version>
    <configuration><classPath>\${project.build.outputDirectory}</classPath></configuration>
    <executions>
      <execution><id>parse</id><phase>generate-sources</phase><goals><goal>parse</goal></goals>
        <configuration><outputDirectory>\${project.build.sourceDirectory}</outputDirectory>
          <classOrPackageName>triton.amd.presets.*</classOrPackageName></configuration></execution>
      <execution><id>build</id><phase>process-classes</phase><goals><goal>build</goal></goals>
        <configuration><classOrPackageName>triton.amd.*</classOrPackageName></configuration></execution>
    </executions>
  </plugin></plugins></build>
</project>
POM
(cd "${WORK}" && mvn -q package)
echo "bindings: ${WORK}/target/tcnative-0.1.0.jar"
