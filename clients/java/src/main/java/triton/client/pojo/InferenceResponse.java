package triton.client.pojo;

import java.util.ArrayList;
import java.util.List;
import java.util.Map;

/** Parsed JSON header of an inference response (reference pojo/InferenceResponse.java). */
public class InferenceResponse {
  private String modelName;
  private String modelVersion;
  private String id;
  private Parameters parameters;
  private List<IOTensor> outputs = new ArrayList<>();

  public InferenceResponse() {}

  public void setModelName(String modelName) { this.modelName = modelName; }

  public void setModelVersion(String modelVersion) { this.modelVersion = modelVersion; }

  public void setId(String id) { this.id = id; }

  public void setParameters(Parameters parameters) { this.parameters = parameters; }

  public void setOutputs(List<IOTensor> outputs) { this.outputs = outputs; }

  public String getModelName() { return modelName; }

  public String getModelVersion() { return modelVersion; }

  public String getId() { return id; }

  public Parameters getParameters() { return parameters; }

  public List<IOTensor> getOutputs() { return outputs; }

  public IOTensor getOutputByName(String name) {
    for (IOTensor t : outputs) {
      if (t.getName().equals(name)) return t;
    }
    return null;
  }

  @SuppressWarnings("unchecked")
  public static InferenceResponse fromJson(Map<String, Object> m) {
    InferenceResponse r = new InferenceResponse();
    r.modelName = (String) m.get("model_name");
    Object v = m.get("model_version");
    r.modelVersion = v == null ? null : v.toString();
    Object id = m.get("id");
    r.id = id == null ? null : id.toString();
    Object p = m.get("parameters");
    if (p instanceof Map) r.parameters = new Parameters((Map<String, Object>) p);
    Object outs = m.get("outputs");
    if (outs instanceof List) {
      for (Object o : (List<Object>) outs) r.outputs.add(IOTensor.fromJson((Map<String, Object>) o));
    }
    return r;
  }
}
