{{- define "voda.image" -}}
{{ .Values.image.repository }}:{{ .Values.image.tag }}
{{- end -}}

{{- define "voda.storeArgs" -}}
"--store", "sqlite:///state/jobs.db", "--mq", "sqlite:///state/mq.db"
{{- end -}}
