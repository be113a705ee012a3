package triton.client.endpoint;

/** A single fixed server address (reference endpoint/FixedEndpoint.java:35-52). */
public class FixedEndpoint extends AbstractEndpoint {
  private final String endpoint;

  public FixedEndpoint(String endpoint) {
    if (endpoint == null || endpoint.isEmpty()) throw new IllegalArgumentException("endpoint is empty");
    this.endpoint = endpoint;
  }

  @Override protected String getEndpointImpl() { return endpoint; }

  @Override public int getEndpointNum() { return 1; }
}
