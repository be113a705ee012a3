package triton.client.pojo;

import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

/** One entry of "inputs"/"outputs" in a request or response (reference pojo/IOTensor.java). */
public class IOTensor {
  private String name;
  private long[] shape;
  private DataType datatype;
  private Parameters parameters;
  private List<Object> data;

  public IOTensor() {}

  public String getName() { return name; }

  public void setName(String name) { this.name = name; }

  public long[] getShape() { return shape; }

  public void setShape(long[] shape) { this.shape = shape; }

  public DataType getDatatype() { return datatype; }

  public void setDatatype(DataType datatype) { this.datatype = datatype; }

  public Parameters getParameters() { return parameters; }

  public void setParameters(Parameters parameters) { this.parameters = parameters; }

  /** JSON "data" (flattened, row-major), or null when the tensor travels as binary. */
  public List<Object> getData() { return data; }

  public void setData(List<Object> data) { this.data = data; }

  /** JSON object form used in the request header. */
  public Map<String, Object> toJson() {
    Map<String, Object> m = new LinkedHashMap<>();
    m.put("name", name);
    if (shape != null) m.put("shape", shape);
    if (datatype != null) m.put("datatype", datatype.name());
    if (parameters != null && !parameters.isEmpty()) m.put("parameters", parameters.asMap());
    if (data != null) m.put("data", data);
    return m;
  }

  @SuppressWarnings("unchecked")
  public static IOTensor fromJson(Map<String, Object> m) {
    IOTensor t = new IOTensor();
    t.name = (String) m.get("name");
    Object shape = m.get("shape");
    if (shape instanceof List) {
      List<Object> s = (List<Object>) shape;
      t.shape = new long[s.size()];
      for (int i = 0; i < s.size(); i++) t.shape[i] = ((Number) s.get(i)).longValue();
    }
    Object dt = m.get("datatype");
    if (dt != null) t.datatype = DataType.valueOf(dt.toString());
    Object p = m.get("parameters");
    if (p instanceof Map) t.parameters = new Parameters((Map<String, Object>) p);
    Object d = m.get("data");
    if (d instanceof List) t.data = Json.flatten((List<Object>) d);
    return t;
  }
}
