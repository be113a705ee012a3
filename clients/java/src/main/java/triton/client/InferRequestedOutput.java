package triton.client;

import triton.client.pojo.IOTensor;
import triton.client.pojo.Parameters;

/** A requested output: binary vs JSON, optional top-k classification (reference InferRequestedOutput.java:36-85). */
public class InferRequestedOutput {
  private final String name;
  private final boolean isBinary;
  private final int classCount;

  public InferRequestedOutput(String name, boolean isBinary, int classCount) {
    Util.checkArgument(!Util.isEmpty(name), "output name must not be empty");
    Util.checkArgument(classCount >= 0, "classCount must be >= 0");
    this.name = name;
    this.isBinary = isBinary;
    this.classCount = classCount;
  }

  public InferRequestedOutput(String name) { this(name, true, 0); }

  public InferRequestedOutput(String name, boolean isBinary) { this(name, isBinary, 0); }

  public String getName() { return name; }

  public boolean isBinary() { return isBinary; }

  public int getClassCount() { return classCount; }

  public IOTensor getTensor() {
    IOTensor t = new IOTensor();
    t.setName(name);
    Parameters p = new Parameters();
    p.put(Parameters.KEY_BINARY_DATA, isBinary);
    if (classCount > 0) p.put(Parameters.KEY_CLASSIFICATION, (long) classCount);
    t.setParameters(p);
    return t;
  }
}
