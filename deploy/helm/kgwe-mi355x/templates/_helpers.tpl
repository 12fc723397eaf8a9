{{- define "kgwe.name" -}}kgwe-mi355x{{- end -}}
{{- define "kgwe.fullname" -}}{{ .Release.Name }}-kgwe{{- end -}}
{{- define "kgwe.image" -}}
{{- $reg := .Values.global.imageRegistry -}}
{{- $tag := default .Chart.AppVersion .Values.image.tag -}}
{{- if $reg }}{{ $reg }}/{{ end }}{{ .Values.image.repository }}:{{ $tag }}
{{- end -}}
{{- define "kgwe.labels" -}}
app.kubernetes.io/name: {{ include "kgwe.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ .Chart.Name }}-{{ .Chart.Version }}
{{- end -}}
{{- define "kgwe.selector" -}}
app.kubernetes.io/name: {{ include "kgwe.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}
